"""Single-image device helpers used off the hot path (writer-side resize)."""
import numpy as np


def resize_area_image(image: np.ndarray, out_h: int, out_w: int) -> np.ndarray:
    """OpenCV INTER_AREA resize of one HWC uint8 image on the HIP device
    (the RRC kernel with a full-image crop); used by RGBImageField's
    ``max_resolution`` (rgb_image.py:37-45)."""
    import torch as ch
    from . import libffcv as L
    if not ch.cuda.is_available():
        raise RuntimeError('max_resolution resizing runs on a HIP device (no CPU fallback)')
    h, w = image.shape[:2]
    dev = ch.device('cuda', ch.cuda.current_device())
    data = ch.from_numpy(np.ascontiguousarray(image).reshape(-1)).to(dev)
    smp = np.zeros(1, L.SAMPLE_DTYPE)
    smp['size'] = image.nbytes
    smp['height'], smp['width'], smp['mode'] = h, w, 1
    d_smp = ch.from_numpy(smp.view(np.uint8)).to(dev)
    crops = ch.tensor([[0, 0, h, w]], dtype=ch.int32, device=dev)
    out = ch.empty((1, out_h, out_w, 3), dtype=ch.uint8, device=dev)
    p = L.RRCParams()
    p.out_h, p.out_w = out_h, out_w
    L.rrc_raw_batch(data, d_smp, 1, crops, None, None, p, out)
    return out[0].cpu().numpy()
