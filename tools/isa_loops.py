"""Instruction mix of the loops of one kernel in a hipcc --save-temps .s:
    python tools/isa_loops.py <file.s> <kernel symbol>
For each loop header label, the straight-line span from the header to the
last branch back to it: counts of VALU / SALU / VMEM / LDS / branch
instructions (a static count: conditional blocks inside count fully)."""
import re
import sys

src, sym = sys.argv[1], sys.argv[2]
lines = open(src).read().split('\n')
start = next(i for i, l in enumerate(lines) if l.startswith(sym + ':'))
end = next(i for i in range(start, len(lines)) if lines[i].startswith('.Lfunc_end'))
body = lines[start:end]
labels = {}
for i, l in enumerate(body):
    m = re.match(r'^(\.LBB\d+_\d+):', l)
    if m:
        labels[m.group(1)] = i
heads = []
for i, l in enumerate(body):
    if 'Loop Header' not in l:
        continue
    j = i
    while j >= 0 and not re.match(r'^\.LBB\d+_\d+:', body[j]):
        j -= 1
    heads.append(re.match(r'^(\.LBB\d+_\d+):', body[j]).group(1))


def kind(ins):
    op = ins.split()[0]
    if op.startswith('v_'):
        return 'valu'
    if op.startswith('s_cbranch') or op.startswith('s_branch'):
        return 'branch'
    if op.startswith('s_waitcnt'):
        return 'wait'
    if op.startswith('s_'):
        return 'salu'
    if op.startswith(('buffer_', 'global_', 'flat_', 'scratch_')):
        return 'vmem'
    if op.startswith('ds_'):
        return 'lds'
    return 'other'


for h in heads:
    i0 = labels[h]
    back = [i for i, l in enumerate(body) if i > i0 and re.search(r's_(c)?branch\w*\s+' + re.escape(h) + r'\b', l)]
    if not back:
        continue
    i1 = back[-1]
    cnt = {}
    for l in body[i0:i1 + 1]:
        t = l.strip()
        if not t or t.startswith(('.', ';')) or t.endswith(':'):
            continue
        k = kind(t)
        cnt[k] = cnt.get(k, 0) + 1
    print(h, f'lines {start + i0 + 1}-{start + i1 + 1}', cnt)
