"""RGB image field and decoders (ffcv/fields/rgb_image.py).

Same classes, constructor arguments and state/allocation semantics as the
reference, but the decoders run on the HIP device that the Loader feeds:

* ``SimpleRGBImageDecoder`` (rgb_image.py:84-139): raw -> device gather,
  jpg -> full JPEG decode kernel; constant-size datasets only (TypeError
  otherwise, as the reference).  Without a GPU (the reference's C1 CPU
  plumbing config) raw samples are copied on the host with ``my_memcpy``.
* ``RandomResizedCropRGBImageDecoder`` / ``CenterCropRGBImageDecoder``
  (rgb_image.py:142-265): crop windows are drawn ON THE DEVICE under the
  per-sample seeding contract (get_random_crop / get_center_crop restated in
  csrc/device_common.h), then one fused kernel decodes only the MCUs the crop
  needs, resizes with OpenCV INTER_AREA semantics and applies any Cutout /
  RandomHorizontalFlip / NormalizeImage that the graph fused into it.

A Loader on ``device='cpu'`` runs the reference's own per-sample host loop
(rgb_image.py:123-136 / 185-210) against the reference-signature C ABI of
libffcv_hip.so: ``imdecode`` (a CPU JPEG decoder with libjpeg-turbo's ifast
+ fancy-upsampling arithmetic, csrc/ffcv_cpu_jpeg.hip, as the reference's
TurboJPEG call), ``resize`` (INTER_AREA on the CPU, the kernels' own
functions) and the contract draws (ffcv_draw_batch_host).  Raw and JPEG
datasets therefore load on a CPU-only machine, as with the reference.
"""
from abc import ABCMeta, abstractmethod
from dataclasses import replace
from typing import Callable, Optional, Tuple, Type

import numpy as np
import torch as ch

from .base import Field, ARG_TYPE
from ..pipeline.operation import Operation
from ..pipeline.state import State
from ..pipeline.allocation_query import AllocationQuery

IMAGE_MODES = {'jpg': 0, 'raw': 1}


def encode_jpeg(numpy_image, quality):
    """rgb_image.py:26-34 (cv2.imencode baseline 4:2:0, standard tables);
    here libjpeg-turbo through Pillow, which emits the same kind of stream."""
    import io
    from PIL import Image
    b = io.BytesIO()
    Image.fromarray(np.ascontiguousarray(numpy_image)).save(b, format='JPEG', quality=int(quality),
                                                            subsampling='4:2:0')
    return np.frombuffer(b.getvalue(), np.uint8).copy()


def resizer(image, target_resolution):
    """rgb_image.py:37-45: shrink so the longest side is target_resolution,
    INTER_AREA (run on the device with the same kernel as the decoders)."""
    if target_resolution is None:
        return image
    original_size = np.array([image.shape[1], image.shape[0]])
    ratio = target_resolution / original_size.max()
    if ratio < 1:
        new_size = (ratio * original_size).astype(int)
        from ..ops import resize_area_image
        image = resize_area_image(image, int(new_size[1]), int(new_size[0]))
    return image


def _pipeline_device(op):
    return getattr(op, '_pipeline_device', None) or ch.device('cpu')


def _host_threads():
    from ..pipeline.compiler import Compiler
    return max(1, int(Compiler.num_threads))


def _raise_failed(L, status, ids):
    bad = np.nonzero(status != 0)[0]
    if bad.size:
        from ..loader.epoch_iterator import DecodeError
        raise DecodeError(f'imdecode failed for sample {int(ids[bad[0]])}: '
                          + L.lib().ffcv_last_error().decode(errors='replace'))


class SimpleRGBImageDecoder(Operation):
    """Most basic decoder for the :class:`~ffcv.fields.RGBImageField`.

    Constant-resolution datasets only; reads (and decompresses) images as is.
    """
    device_aware = True
    per_sample = True

    def __init__(self):
        super().__init__()

    def declare_state_and_memory(self, previous_state: State) -> Tuple[State, AllocationQuery]:
        widths = self.metadata['width']
        heights = self.metadata['height']
        max_width, max_height = widths.max(), heights.max()
        min_height, min_width = heights.min(), widths.min()
        if min_width != max_width or max_height != min_height:
            msg = """SimpleRGBImageDecoder only supports constant image,
consider RandomResizedCropRGBImageDecoder or CenterCropRGBImageDecoder
instead."""
            raise TypeError(msg)
        biggest_shape = (int(max_height), int(max_width), 3)
        dev = _pipeline_device(self)
        self._has_jpg = bool((self.metadata['mode'] == IMAGE_MODES['jpg']).any())
        if dev.type == 'cuda':
            self._on_device = True
            return (replace(previous_state, jit_mode=False, device=dev, shape=biggest_shape,
                            dtype=ch.uint8),
                    (AllocationQuery(biggest_shape, ch.uint8, dev),
                     AllocationQuery((32,), ch.uint8, dev),    # ffcv_sample descriptor
                     AllocationQuery((1,), ch.int32, dev)))    # decode status
        self._on_device = False
        my_dtype = np.dtype('<u1')
        return (replace(previous_state, jit_mode=True, shape=biggest_shape, dtype=my_dtype),
                AllocationQuery(biggest_shape, my_dtype))

    def generate_code(self) -> Callable:
        from .. import libffcv as L
        if not self._on_device:
            mem_read = self.memory_read

            def decode_host(batch_indices, destination, metadata, storage_state):
                # rgb_image.py:123-136 per sample; the raw samples of the batch go
                # through one native gather (ffcv_host_gather) instead of a
                # Python-level read + my_memcpy each (C1: 83 k -> see DESIGN s8)
                B = len(batch_indices)
                fields = metadata[np.asarray(batch_indices, dtype=np.int64)]
                raw = fields['mode'] != IMAGE_MODES['jpg']
                mstate = getattr(storage_state, 'host_state', storage_state)  # BatchContext or the tuple
                if raw.any() and isinstance(mstate, tuple) and len(mstate) in (3, 4) \
                        and isinstance(destination, np.ndarray) and destination.flags['C_CONTIGUOUS']:
                    from ..memory_managers.process_cache import host_source
                    ptrs = fields['data_ptr'][raw].astype(np.uint64)
                    all_ptrs, all_sizes = mstate[1], mstate[2]
                    sizes = all_sizes[np.searchsorted(all_ptrs, ptrs)].astype(np.uint64)
                    row = destination[0].nbytes
                    sizes = np.minimum(sizes, np.uint64(row))
                    src, src_off = host_source(mstate, ptrs)
                    dst_off = np.nonzero(raw)[0].astype(np.uint64) * np.uint64(row)
                    # a thread per 4 MB (the native gather spawns its threads per call)
                    nth = int(min(8, max(1, int(sizes.sum()) >> 22)))
                    L.host_gather(src, src_off, sizes, dst_off, destination, nthreads=nth)
                    todo = np.nonzero(~raw)[0]
                else:
                    todo = range(B)
                todo = np.asarray(todo, np.int64)
                if todo.size:
                    # the remaining samples (JPEG, or raw the gather did not take)
                    # through one native call over the Loader's threads
                    take = set(todo.tolist())
                    images = [mem_read(fields[k]['data_ptr'], storage_state) if k in take else None
                              for k in range(B)]
                    modes = np.full(B, 2, np.uint32)  # 2: skip (gathered above)
                    modes[todo] = np.where(fields['mode'][todo] == IMAGE_MODES['jpg'], 0, 1)
                    status = L.cpu_decode_batch(images, fields['height'], fields['width'], modes, destination[:B],
                                                nthreads=_host_threads())
                    _raise_failed(L, status, np.asarray(batch_indices))
                return destination[:B]
            return decode_host

        f_ix = self._field_index

        def decode(batch_indices, storage, metadata, ss):
            out, smp, status = storage
            B = len(batch_indices)
            stream = ss.stream
            samples = ss.batch_samples(f_ix, smp)
            stride = out[0].numel()
            if ss.any_mode(f_ix, 1):
                L.gather_raw_batch(ss.data, samples, B, out, stride, stream)
            if ss.any_mode(f_ix, 0):
                dec = ss.jpeg_decoder(f_ix)
                dec.decode(ss.data, samples, B, out, stride, status, stream)
                ss.check_status(status[:B], 'SimpleRGBImageDecoder')
            return out[:B]
        return decode


class ResizedCropRGBImageDecoder(SimpleRGBImageDecoder, metaclass=ABCMeta):
    """Abstract crop-then-resize decoder (rgb_image.py:142-217)."""

    crop_kind = 0

    def __init__(self, output_size):
        super().__init__()
        self.output_size = output_size
        self._fused_cutout = None
        self._fused_flip = None
        self._cutout_before_flip = False
        self._fused_normalize = None

    # graph lowering hooks -------------------------------------------------
    def fuse(self, cutout=None, flip=None, cutout_before_flip=False, normalize=None):
        self._fused_cutout = cutout
        self._fused_flip = flip
        self._cutout_before_flip = cutout_before_flip
        self._fused_normalize = normalize

    @property
    def output_dtype(self):
        return ch.float16 if self._fused_normalize is not None else ch.uint8

    def declare_state_and_memory(self, previous_state: State) -> Tuple[State, AllocationQuery]:
        widths = self.metadata['width']
        heights = self.metadata['height']
        self.max_width = np.uint64(widths.max())
        self.max_height = np.uint64(heights.max())
        dev = _pipeline_device(self)
        output_shape = (int(self.output_size[0]), int(self.output_size[1]), 3)
        self._on_device = dev.type == 'cuda'
        if not self._on_device:  # rgb_image.py:151-166: output + full-image temp per sample
            u1 = np.dtype('<u1')
            return (replace(previous_state, jit_mode=True, shape=output_shape, dtype=u1),
                    (AllocationQuery(output_shape, u1),
                     AllocationQuery((int(self.max_height) * int(self.max_width) * 3,), u1)))
        return (
            replace(previous_state, jit_mode=False, device=dev, shape=output_shape,
                    dtype=self.output_dtype),
            (AllocationQuery(output_shape, self.output_dtype, dev),
             AllocationQuery((32,), ch.uint8, dev),  # ffcv_sample descriptor
             AllocationQuery((4,), ch.int32, dev),   # crop window
             AllocationQuery((2,), ch.int32, dev),   # cutout origin
             AllocationQuery((1,), ch.uint8, dev),   # flip decision
             AllocationQuery((1,), ch.int32, dev)),  # decode status
        )

    def _draw_params(self, ss, out_h, out_w):
        key = (int(ss.loader_seed), int(ss.epoch), out_h, out_w)
        cached = getattr(self, '_dp_cache', None)
        if cached is not None and cached[0] == key:
            return cached[1]
        p = self._make_draw_params(ss, out_h, out_w)
        self._dp_cache = (key, p)
        return p

    def _make_draw_params(self, ss, out_h, out_w):
        from .. import libffcv as L
        p = L.DrawParams()
        p.crop_kind = self.crop_kind
        p.out_h, p.out_w = out_h, out_w
        if self.crop_kind == 0:
            p.scale[0], p.scale[1] = float(self.scale[0]), float(self.scale[1])
            p.ratio[0], p.ratio[1] = float(self.ratio[0]), float(self.ratio[1])
        else:
            p.center_ratio = float(self.ratio)
        p.cutout_size = int(self._fused_cutout.crop_size) if self._fused_cutout is not None else 0
        if self._fused_flip is not None:
            p.flip_prob = float(self._fused_flip.flip_prob)
        p.loader_seed = int(ss.loader_seed) & 0xFFFFFFFFFFFFFFFF
        p.epoch = int(ss.epoch)
        return p

    def _generate_code_host(self) -> Callable:
        """The reference's per-sample loop (rgb_image.py:185-210) on host
        buffers through the C ABI (imdecode / draws / resize)."""
        from .. import libffcv as L
        from ..pipeline import runtime
        mem_read = self.memory_read
        jpg = IMAGE_MODES['jpg']

        def decode(batch_indices, my_storage, metadata, storage_state):
            destination, temp_storage = my_storage
            B = len(batch_indices)
            ids = np.asarray(batch_indices, dtype=np.uint64)
            fields = metadata[ids.astype(np.int64)]
            ctx = runtime.current()
            seed, epoch = (ctx.loader_seed, ctx.epoch) if ctx is not None else (0, 0)
            out_h, out_w = int(destination.shape[1]), int(destination.shape[2])
            dp = self._make_draw_params_seed(seed, epoch, out_h, out_w)
            crops = np.empty((B, 4), np.int32)
            L.draw_batch_host(ids, fields['height'], fields['width'], dp, crops)
            # imdecode -> crop -> resize per sample, the reference's prange loop
            # (rgb_image.py:185-210) as one native call over the Loader's threads
            images = [mem_read(f['data_ptr'], storage_state) for f in fields]
            modes = np.where(fields['mode'] == jpg, 0, 1)
            dst = destination[:B]
            status = L.cpu_decode_batch(images, fields['height'], fields['width'], modes, dst, crops,
                                        nthreads=_host_threads())
            _raise_failed(L, status, ids)
            return dst
        decode.is_parallel = True
        return decode

    def _make_draw_params_seed(self, seed, epoch, out_h, out_w):
        class _S:
            pass
        ss = _S()
        ss.loader_seed, ss.epoch = seed, epoch
        p = self._make_draw_params(ss, out_h, out_w)
        p.cutout_size = 0  # host Cutout / flip run as their own operations
        p.flip_prob = 0.0
        return p

    def generate_code(self) -> Callable:
        from .. import libffcv as L
        if not getattr(self, '_on_device', True):
            return self._generate_code_host()
        f_ix = self._field_index
        rp = L.RRCParams()
        cut = self._fused_cutout
        if cut is not None:
            rp.cutout_size = int(cut.crop_size)
            fill = np.asarray(cut.fill).astype(np.uint8).reshape(-1)
            fill = np.broadcast_to(fill, (3,)) if fill.size == 1 else fill
            for i in range(3):
                rp.cutout_fill[i] = int(fill[i])
            rp.cutout_fill[3] = int(self._cutout_before_flip)
        norm = self._fused_normalize
        use_flip = self._fused_flip is not None

        def decode(batch_indices, storage, metadata, ss):
            out, smp, crops, cyx, flips, status = storage
            B = len(batch_indices)
            stream = ss.stream
            # the target size is the destination's, like the reference's
            # resize_crop(..., destination[dst_ix]) (rgb_image.py:207-208):
            # a new output_size between epochs gets new buffers and is used
            rp.out_h, rp.out_w = int(out.shape[1]), int(out.shape[2])
            dp = self._draw_params(ss, rp.out_h, rp.out_w)
            if norm is not None:
                rp.lut = norm.device_lut(out.device).data_ptr()
            rp.out_stride = out[0].numel() * out.element_size()
            if ss.dataset.data is not None and ss.any_mode(f_ix, 0):
                # HBM-resident dataset: gather + draws run inside the entropy
                # kernel (ffcv_jpeg_rrc_fused), two fewer launches per batch
                dec = ss.jpeg_decoder(f_ix)
                dec.rrc_fused(ss.data, ss.sample_table(f_ix), ss.batch_ids, dp, crops,
                              cyx if cut is not None else None, flips if use_flip else None, rp, out,
                              status, samples_out=smp, stream=stream)
                ss.check_status(status[:B], type(self).__name__)
                if ss.any_mode(f_ix, 1):
                    L.rrc_raw_batch(ss.data, smp[:B], B, crops, cyx if cut is not None else None,
                                    flips if use_flip else None, rp, out, stream,
                                    workspace=ss.raw_workspace(f_ix, rp.out_h, rp.out_w))
                return out[:B]
            samples = ss.batch_samples(f_ix, smp)
            L.draw_batch(ss.batch_ids, samples, dp, crops, cyx if cut is not None else None,
                         flips if use_flip else None, None, stream)
            if ss.any_mode(f_ix, 1):
                L.rrc_raw_batch(ss.data, samples, B, crops, cyx if cut is not None else None,
                                flips if use_flip else None, rp, out, stream,
                                workspace=ss.raw_workspace(f_ix, rp.out_h, rp.out_w))
            if ss.any_mode(f_ix, 0):
                dec = ss.jpeg_decoder(f_ix)
                dec.rrc(ss.data, samples, B, crops, cyx if cut is not None else None,
                        flips if use_flip else None, rp, out, status, stream)
                ss.check_status(status[:B], type(self).__name__)
            return out[:B]
        return decode

    @property
    @abstractmethod
    def get_crop_generator(self):
        raise NotImplementedError


class RandomResizedCropRGBImageDecoder(ResizedCropRGBImageDecoder):
    """Random crop + resize (rgb_image.py:220-242): ``output_size`` is the
    (height, width) every crop is resized to; a crop's area is a fraction
    of the image drawn from ``scale`` and its width/height from ``ratio``
    (log-uniform), torchvision's RandomResizedCrop rule (get_random_crop)."""
    crop_kind = 0

    def __init__(self, output_size, scale=(0.08, 1.0), ratio=(0.75, 4 / 3)):
        super().__init__(output_size)
        self.scale = scale
        self.ratio = ratio
        self.output_size = output_size

    @property
    def get_crop_generator(self):
        return 'get_random_crop'


class CenterCropRGBImageDecoder(ResizedCropRGBImageDecoder):
    """Center crop + resize (rgb_image.py:245-265); ratio = crop / min side."""
    crop_kind = 1

    def __init__(self, output_size, ratio):
        super().__init__(output_size)
        self.scale = None
        self.ratio = ratio

    @property
    def get_crop_generator(self):
        return 'get_center_crop'


class RGBImageField(Field):
    """RGB image field (rgb_image.py:268-365).

    Parameters
    ----------
    write_mode : str, optional
        'raw', 'jpg', 'smart' or 'proportion'. By default: 'raw'.
    max_resolution : int, optional
        If specified, resize images so the longest side is this value.
    smart_threshold : int, optional
        When `write_mode='smart`, compress images whose raw size exceeds this.
    jpeg_quality : int, optional
        JPEG quality (ignored for raw), by default 90.
    compress_probability : float, optional
        Probability of JPEG compression for write_mode='proportion'.
    """

    def __init__(self, write_mode='raw', max_resolution: int = None, smart_threshold: int = None,
                 jpeg_quality: int = 90, compress_probability: float = 0.5) -> None:
        self.write_mode = write_mode
        self.smart_threshold = smart_threshold
        self.max_resolution = max_resolution
        self.jpeg_quality = int(jpeg_quality)
        self.proportion = compress_probability

    @property
    def metadata_type(self) -> np.dtype:
        return np.dtype([('mode', '<u1'), ('width', '<u2'), ('height', '<u2'), ('data_ptr', '<u8')])

    def get_decoder_class(self) -> Type[Operation]:
        return SimpleRGBImageDecoder

    @staticmethod
    def from_binary(binary: ARG_TYPE) -> Field:
        return RGBImageField()

    def to_binary(self) -> ARG_TYPE:
        return np.zeros(1, dtype=ARG_TYPE)[0]

    def encode(self, destination, image, malloc):
        try:
            from PIL.Image import Image
            if isinstance(image, Image):
                image = np.array(image)
        except ImportError:
            pass
        if not isinstance(image, np.ndarray):
            raise TypeError(f"Unsupported image type {type(image)}")
        if image.dtype != np.uint8:
            raise ValueError("Image type has to be uint8")
        if image.shape[2] != 3:
            raise ValueError(f"Invalid shape for rgb image: {image.shape}")
        image = resizer(image, self.max_resolution)
        write_mode = self.write_mode
        as_jpg = None
        if write_mode == 'smart':
            as_jpg = encode_jpeg(image, self.jpeg_quality)
            write_mode = 'raw'
            if self.smart_threshold is not None:
                if image.nbytes > self.smart_threshold:
                    write_mode = 'jpg'
        elif write_mode == 'proportion':
            if np.random.rand() < self.proportion:
                write_mode = 'jpg'
            else:
                write_mode = 'raw'
        destination['mode'] = IMAGE_MODES[write_mode]
        destination['height'], destination['width'] = image.shape[:2]
        if write_mode == 'jpg':
            if as_jpg is None:
                as_jpg = encode_jpeg(image, self.jpeg_quality)
            destination['data_ptr'], storage = malloc(as_jpg.nbytes)
            storage[:] = as_jpg
        elif write_mode == 'raw':
            image_bytes = np.ascontiguousarray(image).view('<u1').reshape(-1)
            destination['data_ptr'], storage = malloc(image.nbytes)
            storage[:] = image_bytes
        else:
            raise ValueError(f"Unsupported write mode {self.write_mode}")
