"""Code-generation guards on the built gfx950 code object (no GPU needed).

jpeg_rrc_loop_kernel<true> (ffcv_jpeg.hip, K2L) waits for the next band's
plane tiles, copied HBM -> LDS by global_load_lds, with a counted
``s_waitcnt vmcnt(half)``: the walk issues exactly one 12-byte output store
per row after those loads, and vmcnt retires in order, so once at most `half`
operations are outstanding the tile loads have landed.  That holds only while
the compiler keeps the store unconditional in the walk loop's latch (ADVICE
r4).  This test reads the disassembly of the library the product loads."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = '/opt/rocm/lib/llvm/bin'
LIB = os.path.join(ROOT, 'ffcv_amd', 'libffcv_hip.so')
HALF = 8  # jpeg_rrc_loop_kernel: rows per row group (BAND 16 / 2 row groups)


def _disassemble():
    bundler, objdump = os.path.join(LLVM, 'clang-offload-bundler'), os.path.join(LLVM, 'llvm-objdump')
    if not (os.path.exists(bundler) and os.path.exists(objdump) and shutil.which('objcopy')):
        pytest.skip('ROCm LLVM tools / objcopy not available')
    from ffcv_amd import _build
    _build.build()
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        fat = os.path.join(d, 'fat.bin')
        subprocess.check_call(['objcopy', '-O', 'binary', '--only-section=.hip_fatbin', LIB, fat])
        data = open(fat, 'rb').read()
        magic = b'__CLANG_OFFLOAD_BUNDLE__'
        offs = [m.start() for m in re.finditer(re.escape(magic), data)]
        text = []
        for n, (a, b) in enumerate(zip(offs, offs[1:] + [len(data)])):
            part, co = os.path.join(d, f'b{n}.bin'), os.path.join(d, f'c{n}.co')
            open(part, 'wb').write(data[a:b])
            subprocess.check_call([bundler, '--unbundle', '--type=o', '--targets=hipv4-amdgcn-amd-amdhsa--gfx950',
                                   f'--input={part}', f'--output={co}'])
            text.append(subprocess.run([objdump, '-d', '--mcpu=gfx950', co], capture_output=True, text=True,
                                       check=True).stdout)
    return '\n'.join(text)


def _kernel(asm, mangled):
    lines = asm.splitlines()
    st = [i for i, l in enumerate(lines) if l.endswith('>:') and mangled in l]
    assert len(st) == 1, f'{mangled}: {len(st)} symbols'
    en = next((i for i in range(st[0] + 1, len(lines)) if lines[i].endswith('>:')), len(lines))
    return [l.split('//')[0].strip() for l in lines[st[0] + 1:en] if l.strip()]


def test_k2_loop_walk_store_count_matches_vmcnt():
    asm = _disassemble()
    body = _kernel(asm, '_Z20jpeg_rrc_loop_kernelILb1EEv8JpegArgs')
    assert any(l == f's_waitcnt vmcnt({HALF})' for l in body), 'the counted tile wait is gone'
    stores = [i for i, l in enumerate(body) if l.startswith('global_store_dwordx3') and l.endswith(' nt')]
    lds = [j for j, l in enumerate(body) if l.startswith('global_load_lds')]
    assert stores and lds
    # the band walk's store: the first streaming store after the tile loads
    # (the general path's k2_band walk, inlined too, has its own)
    after = [i for i in stores if i > lds[-1]]
    assert after, 'no walk store after the tile loads'
    i = after[0]
    # the store sits in the walk loop's latch block: the next control-flow
    # instruction is the loop's conditional exit test, with no other memory
    # operation or branch in between -- so every walk row issues exactly one
    # vector-memory instruction after the band's tile loads
    for l in body[i + 1:i + 12]:
        op = l.split()[0]
        if op.startswith('s_cbranch_scc'):
            break
        assert not op.startswith(('s_cbranch', 's_branch', 'global_', 'buffer_', 'flat_', 's_setpc')), l
    else:
        raise AssertionError('no loop-exit test right after the walk store')
    # and no other vector-memory instruction (loads included) between the
    # band's last tile load and the walk store
    between = [l for l in body[lds[-1] + 1:i] if l.split()[0].startswith(('global_', 'buffer_', 'flat_'))]
    assert not between, between
