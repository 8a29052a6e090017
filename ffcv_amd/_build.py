"""Build ``ffcv_amd/libffcv_hip.so`` for gfx950 in-tree (hipcc).

    python -m ffcv_amd._build [--force]

The .so is git-ignored but travels to the GPU box with the gpurun snapshot.
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, 'csrc')
OUT = os.path.join(HERE, 'libffcv_hip.so')
SOURCES = ['ffcv_common.hip', 'ffcv_rrc.hip', 'ffcv_jpeg.hip', 'ffcv_host.hip', 'ffcv_cpu_jpeg.hip']
HEADERS = ['api_internal.h', 'device_common.h', 'diag_hooks.h']
ARCH = os.environ.get('PYTORCH_ROCM_ARCH', 'gfx950').split(';')[0]

FLAGS = ['--offload-arch=' + ARCH, '-O3', '-fPIC', '-shared', '-std=c++17',
         # bit-exact float paths (INTER_AREA taps, crop draws): no FMA contraction
         '-ffp-contract=off', '-fno-fast-math', '-Wall', '-Wno-unused-function']


def _stale():
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    deps = [os.path.join(CSRC, f) for f in SOURCES + HEADERS]
    deps.append(os.path.join(os.path.dirname(HERE), 'include', 'ffcv_hip.h'))
    return any(os.path.getmtime(d) > t for d in deps)


def build(force=False, verbose=False):
    if not force and not _stale():
        return OUT
    hipcc = os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')
    cmd = [hipcc] + FLAGS + ['-o', OUT + '.tmp'] + [os.path.join(CSRC, s) for s in SOURCES]
    if verbose:
        print(' '.join(cmd))
    subprocess.check_call(cmd, cwd=CSRC)
    os.replace(OUT + '.tmp', OUT)
    return OUT


if __name__ == '__main__':
    print(build(force='--force' in sys.argv, verbose=True))
