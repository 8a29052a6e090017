"""Per-sample seeding contract shared by the host paths of the transforms.

Each stochastic operation ``op`` applied to dataset sample ``s`` in epoch
``e`` of a Loader seeded with ``seed`` owns a fresh MT19937 seeded with
``low32(splitmix64(splitmix64(splitmix64(seed ^ op<<56) ^ e) ^ s))``;
op ids: 1 crop, 2 cutout, 3 flip.  The device kernels use the same function
(csrc/device_common.h sample_seed).  The reference itself draws from numba's
per-thread generators seeded from OS entropy (nondeterministic); see
DESIGN.md "RNG contract".
"""
M64 = (1 << 64) - 1


def splitmix64(x):
    z = (x + 0x9E3779B97F4A7C15) & M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def contract_seed(loader_seed, epoch, sample, op_id):
    h = splitmix64((int(loader_seed) & M64) ^ ((int(op_id) << 56) & M64))
    h = splitmix64(h ^ (int(epoch) & M64))
    h = splitmix64(h ^ (int(sample) & M64))
    return h & 0xFFFFFFFF
