from .cutout import Cutout
from .flip import RandomHorizontalFlip
from .ops import ToTensor, ToDevice, ToTorchImage, Convert, View
from .normalize import NormalizeImage
from .module import ModuleWrapper
from .common import Squeeze

__all__ = ['ToTensor', 'ToDevice', 'ToTorchImage', 'NormalizeImage', 'Convert', 'Squeeze', 'View',
           'RandomHorizontalFlip', 'Cutout', 'ModuleWrapper']
