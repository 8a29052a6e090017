"""cProfile of the Loader's producer thread in device_cache mode (host-side
cost per batch).  python tools/loader_profile.py [n] -> gpurun_out/loader_prof.txt"""
import cProfile
import io
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402



def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
    import subprocess
    d = '/tmp/lp'
    os.makedirs(d, exist_ok=True)
    fn = os.path.join(d, f'loader_bench_{n}.beton')
    if not os.path.exists(fn):
        subprocess.check_call([sys.executable, 'tools/loader_bench.py', '--n', str(n), '--epochs', '1',
                               '--dir', d, '--modes', 'device_cache'])
    from bench import IMAGENET_MEAN, IMAGENET_STD
    from ffcv_amd.fields.decoders import RandomResizedCropRGBImageDecoder, IntDecoder
    from ffcv_amd.transforms import ToTensor, ToDevice, ToTorchImage, NormalizeImage, Cutout
    from ffcv_amd.loader import Loader, OrderOption
    import ffcv_amd.loader.epoch_iterator as EI
    dev = torch.device('cuda:0')
    loader = Loader(fn, batch_size=512, order=OrderOption.RANDOM, seed=0, drop_last=True, device=dev,
                    pipelines={'image': [RandomResizedCropRGBImageDecoder((224, 224)), Cutout(32, (124, 116, 103)),
                                         ToTensor(), ToDevice(dev), ToTorchImage(),
                                         NormalizeImage(IMAGENET_MEAN, IMAGENET_STD, np.float16)],
                               'label': [IntDecoder(), ToTensor(), ToDevice(dev)]})
    for _ in loader:
        pass
    torch.cuda.synchronize()
    prof = cProfile.Profile()
    orig = EI.EpochIterator.run

    def run(self):
        prof.enable()
        try:
            orig(self)
        finally:
            prof.disable()
    EI.EpochIterator.run = run
    t0 = time.perf_counter()
    nb = 0
    for _ in range(3):
        for _ in loader:
            nb += 1
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    s = io.StringIO()
    print(f'{nb} batches, {el * 1e3 / nb:.3f} ms/batch (profiled), {nb * 512 / el:.0f} img/s', file=s)
    pstats.Stats(prof, stream=s).sort_stats('tottime').print_stats(35)
    os.makedirs('gpurun_out', exist_ok=True)
    open('gpurun_out/loader_prof.txt', 'w').write(s.getvalue())
    print(s.getvalue()[:3000])


if __name__ == '__main__':
    main()
