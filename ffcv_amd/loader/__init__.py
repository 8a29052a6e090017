from .loader import Loader, OrderOption

__all__ = ['Loader', 'OrderOption']
