"""Single-image helpers used off the hot path (writer-side resize)."""
import numpy as np


def resize_area_image(image: np.ndarray, out_h: int, out_w: int) -> np.ndarray:
    """cv2.resize(image, (out_w, out_h), interpolation=INTER_AREA) of one HWC
    uint8 image, as RGBImageField's ``max_resolution`` does at write time
    (rgb_image.py:37-45).  Runs the C-ABI ``resize`` of libffcv_hip.so on the
    host (the kernels' own INTER_AREA functions compiled for the CPU), so
    writing a dataset needs no GPU."""
    from . import libffcv as L
    src = np.ascontiguousarray(image, dtype=np.uint8)
    out = np.empty((int(out_h), int(out_w), 3), np.uint8)
    L.resize_crop(src, 0, src.shape[0], 0, src.shape[1], out)
    return out
