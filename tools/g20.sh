for rep in 1 2; do for g in 12 7 5 10; do
timeout -k 10 120 python bench.py --steps 20 --warmup 5 --group $g --no-cpu-baseline > gpurun_out/g20_$g.log 2>&1 || exit 1
python -c "import json;d=json.loads(open('gpurun_out/g20_$g.log').read().strip().splitlines()[-1]);print('group $g', d['value'], d['roofline']['launches'])"
done; done
