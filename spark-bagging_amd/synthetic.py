"""Host twin of the device generator k_synth (sbag_kernels.hip) for the synthetic
bench workload: x[r,f] = splitmix64(seed ^ (r*F+f)) mod 32,
regression label k = sum_{f<8} (f+1) x[r,f] + (h2 mod 64) - 32, y = k / 64,
class label (x0 + 3 x1 + 7 x2 + h2 mod 8) mod C, h2 = splitmix64(~seed ^ r).
"""
import numpy as np

M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def splitmix64(z):
    z = np.asarray(z, np.uint64)
    with np.errstate(over="ignore"):
        z = z + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def generate(num_rows, num_features, seed=20261015, num_classes=0, row_begin=0):
    rows = np.arange(row_begin, row_begin + num_rows, dtype=np.uint64)
    idx = rows[:, None] * np.uint64(num_features) + np.arange(num_features, dtype=np.uint64)[None, :]
    x = (splitmix64(np.uint64(seed) ^ idx) & np.uint64(31)).astype(np.int64)
    h2 = splitmix64((np.uint64(seed) ^ M64) ^ rows)
    if num_classes == 0:
        k = np.zeros(num_rows, np.int64)
        for f in range(min(8, num_features)):
            k += (f + 1) * x[:, f]
        k += (h2 & np.uint64(63)).astype(np.int64) - 32
        y = np.ldexp(k.astype(np.float64), -6)
    else:
        y = ((x[:, 0] + 3 * x[:, 1] + 7 * x[:, 2] + (h2 & np.uint64(7)).astype(np.int64))
             % num_classes).astype(np.float64)
    return x.astype(np.float64), y
