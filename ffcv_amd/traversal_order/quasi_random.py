"""ffcv/traversal_order/quasi_random.py:15-85: page-local shuffle that limits
disk reads when the dataset does not fit in RAM.  With the dataset resident
in HBM it buys nothing, and the reference does not support it distributed
(quasi_random.py:54-56).  Implemented on the host (index generation only):
shuffle samples inside each page, visit pages in a random order keeping a
window of ``2*batch_size`` open pages, seed ``seed*912300 + epoch``."""
from typing import Sequence

import numpy as np

from .base import TraversalOrder


class QuasiRandom(TraversalOrder):

    def __init__(self, loader):
        super().__init__(loader)
        self.page_to_samples = loader.memory_manager.page_to_samples
        if not self.page_to_samples:
            raise ValueError("Dataset won't benefit from QuasiRandom order, use regular Random")
        if self.distributed:
            raise NotImplementedError("distributed Not implemented yet for QuasiRandom")
        index_set = set(int(i) for i in self.indices)
        self.pages = {int(p): sorted(int(s) for s in v if int(s) in index_set)
                      for p, v in self.page_to_samples.items()}

    def sample_order(self, epoch: int) -> Sequence[int]:
        rng = np.random.default_rng(self.seed * 912300 + epoch)
        pages = [np.array(v, np.int64) for _, v in sorted(self.pages.items()) if v]
        for p in pages:
            rng.shuffle(p)
        order = rng.permutation(len(pages))
        window = max(1, 2 * self.loader.batch_size)
        result, open_pages, consumed, nxt = [], [], {}, 0
        total = sum(len(p) for p in pages)
        while len(result) < total:
            while nxt < len(order) and len(open_pages) < window:
                open_pages.append(int(order[nxt]))
                consumed[int(order[nxt])] = 0
                nxt += 1
            k = int(rng.integers(0, len(open_pages)))
            pg = open_pages[k]
            result.append(pages[pg][consumed[pg]])
            consumed[pg] += 1
            if consumed[pg] >= len(pages[pg]):
                open_pages.pop(k)
        return np.array(result, dtype=np.int64)
