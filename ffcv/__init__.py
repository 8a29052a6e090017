"""The ``ffcv`` import name of this framework (drop-in for libffcv/ffcv).

User code written for the reference keeps its imports unchanged::

    from ffcv.loader import Loader, OrderOption
    from ffcv.fields import RGBImageField, IntField
    from ffcv.fields.decoders import RandomResizedCropRGBImageDecoder
    from ffcv.transforms import ToTensor, ToDevice, ToTorchImage, Cutout
    from ffcv.writer import DatasetWriter

Every ``ffcv.<path>`` module is the same module object as
``ffcv_amd.<path>`` (a meta-path finder aliases them; nothing is copied),
so classes and isinstance checks agree between the two names.  Fields the
reference keeps in their own modules map to where this package defines
them (NDArray / TorchTensor / JSON descriptors live in
``ffcv_amd.fields.unsupported``).
"""
import importlib
import importlib.abc
import importlib.util
import sys

_IMPL = 'ffcv_amd'
_RENAMED = {
    'ffcv.fields.ndarray': 'ffcv_amd.fields.unsupported',
    'ffcv.fields.json': 'ffcv_amd.fields.unsupported',
}


def _target(fullname):
    if fullname in _RENAMED:
        return _RENAMED[fullname]
    return _IMPL + fullname[len('ffcv'):]


class _AliasFinder(importlib.abc.MetaPathFinder, importlib.abc.Loader):
    def find_spec(self, fullname, path, target=None):
        if not fullname.startswith('ffcv.'):
            return None
        real = _target(fullname)
        try:
            spec = importlib.util.find_spec(real)
        except ModuleNotFoundError:
            return None
        if spec is None:
            return None
        return importlib.util.spec_from_loader(fullname, self,
                                               is_package=spec.submodule_search_locations is not None)

    def create_module(self, spec):
        # the implementation module itself: one module object, two names
        return importlib.import_module(_target(spec.name))

    def exec_module(self, module):
        pass


if not any(isinstance(f, _AliasFinder) for f in sys.meta_path):
    sys.meta_path.insert(0, _AliasFinder())

_impl = importlib.import_module(_IMPL)
Loader = _impl.Loader
DatasetWriter = _impl.DatasetWriter
__version__ = _impl.__version__
__all__ = ['Loader']
