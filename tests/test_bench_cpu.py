"""bench.py's host logic that needs no GPU: the --gpus N self-launch
 and the launch split."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_self_launch_cmd_shape():
    cmd = bench.self_launch_cmd(['--gpus', '8', '--steps', '20', '--warmup', '5'], 8, 29999)
    assert cmd[:3] == [sys.executable, '-m', 'torch.distributed.run']
    i = cmd.index('--nproc-per-node')
    assert cmd[i + 1] == '8'
    assert cmd[cmd.index('--master-addr') + 1] == '127.0.0.1'
    assert cmd[cmd.index('--master-port') + 1] == '29999'
    j = cmd.index(os.path.join(ROOT, 'bench.py'))
    assert cmd[j + 1:] == ['--gpus', '8', '--steps', '20', '--warmup', '5']


def test_gpus_n_spawns_ranks_and_propagates_failure():
    """`bench.py --gpus 2` outside torchrun starts torchrun as a child with
    two ranks, each of which re-enters bench.py (here each rank fails its own
    argument parsing on purpose, before touching any device), and the
    launcher exits non-zero with the ranks' errors on stderr."""
    env = {k: v for k, v in os.environ.items() if k not in ('RANK', 'WORLD_SIZE', 'LOCAL_RANK')}
    r = subprocess.run([sys.executable, os.path.join(ROOT, 'bench.py'), '--gpus', '2', '--config', 'nope'],
                       capture_output=True, text=True, timeout=120, env=env, cwd=ROOT)
    assert r.returncode != 0
    assert 'torch.distributed.run' in r.stderr and '--nproc-per-node 2' in r.stderr
    # both ranks ran bench.py's full argument parser
    assert r.stderr.count("invalid choice: 'nope'") >= 2, r.stderr[-2000:]


def test_rank_count_must_match_gpus():
    """Under a launcher, --gpus must equal the world size the launcher
    started (the driver's `torchrun --nproc-per-node N bench.py --gpus N`)."""
    env = dict(os.environ, RANK='0', WORLD_SIZE='1', LOCAL_RANK='0')
    r = subprocess.run([sys.executable, os.path.join(ROOT, 'bench.py'), '--gpus', '2'],
                       capture_output=True, text=True, timeout=120, env=env, cwd=ROOT)
    assert r.returncode != 0 and 'launcher started 1 ranks' in r.stderr
