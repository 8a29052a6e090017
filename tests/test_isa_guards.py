"""Code-generation guards on the built gfx950 code object (no GPU needed).

The hot kernels are tuned to their register budgets (K1 at 4 waves per SIMD,
K2 at 6, K1b and the raw kernel at theirs): a source change that makes the
compiler spill vector registers to scratch memory costs 5-30% without any
wrong pixel (the C5 staging arrays moved to scratch ran 2.28 M
vs 2.95 M).  These tests read the disassembly of the library the product
loads and fail on any scratch access in those kernels.  (Round 6: the
band-loop K2 and its counted-vmcnt guard were deleted.)"""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = '/opt/rocm/lib/llvm/bin'
LIB = os.path.join(ROOT, 'ffcv_amd', 'libffcv_hip.so')


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


HOT = ['_Z19jpeg_entropy_kernelILi0EEv8JpegArgs',            # K1 (RRC)
       '_Z16jpeg_idct_kernel8JpegArgs',                        # K1b
       '_Z24jpeg_color_resize_kernelILi0ELb1EEv8JpegArgs',     # K2, fp16 LUT
       '_Z24jpeg_color_resize_kernelILi0ELb0EEv8JpegArgs',     # K2, u8
       '_Z14rrc_raw_kernelILb0EEv']                            # C5 raw kernel (prefix)


def test_hot_kernels_do_not_spill_to_scratch():
    asm = _disassemble()
    for m in HOT:
        body = _kernel(asm, m)
        bad = [l for l in body if l.split()[0].startswith('scratch_')]
        assert not bad, f'{m}: {len(bad)} scratch accesses, e.g. {bad[:3]}'


def test_band_loop_kernel_is_gone():
    asm = _disassemble()
    assert 'jpeg_rrc_loop_kernel' not in asm
