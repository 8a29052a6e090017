"""Per-basic-block instruction counts of one loop (by header label) in a
kernel's .s extract:  python tools/isa_loop_blocks.py <k.s> <header label>
Blocks are attributed to the loop by LLVM's 'in Loop: Header=' comments."""
import sys

src, head = sys.argv[1], sys.argv[2].lstrip('.L')
lines = open(src).read().split('\n')
blocks, order, cur, inloop = {}, [], None, False
for i, l in enumerate(lines):
    if l.startswith('.LBB') or l.startswith('; %bb'):
        nxt = lines[i + 1] if i + 1 < len(lines) else ''
        cur = l.split(':')[0]
        inloop = f'Header={head} ' in l + ' ' or f'Header={head} ' in nxt + ' ' or l.startswith(f'.L{head}:')
        if inloop and cur not in blocks:
            blocks[cur] = {}
            order.append(cur)
        continue
    t = l.strip()
    if not inloop or not t or t.startswith(('.', ';')):
        continue
    op = t.split()[0]
    k = ('valu' if op.startswith('v_') else 'branch' if 'branch' in op else 'wait' if 'waitcnt' in op else
         'salu' if op.startswith('s_') else 'vmem' if op.startswith(('buffer', 'global', 'flat')) else
         'lds' if op.startswith('ds_') else 'other')
    blocks[cur][k] = blocks[cur].get(k, 0) + 1
tot = {}
for b in order:
    print(b, blocks[b])
    for k, v in blocks[b].items():
        tot[k] = tot.get(k, 0) + v
print('total', tot)
