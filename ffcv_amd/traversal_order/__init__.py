from .sequential import Sequential
from .random import Random
from .quasi_random import QuasiRandom

__all__ = ['Sequential', 'Random', 'QuasiRandom']
