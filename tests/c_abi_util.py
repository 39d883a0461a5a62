"""Helpers for the plain-C driver tests/c/abi_driver (the JNI shim's argument order)."""
import os
import struct
import subprocess

import numpy as np

from conftest import ROOT

DRIVER = os.path.join(ROOT, "tests", "c", "abi_driver")
DRIVER_ASAN = os.path.join(ROOT, "tests", "c", "abi_driver_asan")


def run_driver(tmp_path, X, y, offsets, *, replacement, ratio, seed, lb, le, sub_ratio,
               bug_compat, depth, bins, min_inst, impurity, min_gain, tree_seed, agg,
               driver=DRIVER, env=None):
    X = np.ascontiguousarray(X, np.float64)
    y = np.ascontiguousarray(y, np.float64)
    off = np.asarray(offsets, np.int64)
    data = tmp_path / "data.bin"
    out = tmp_path / "out.bin"
    with open(data, "wb") as f:
        f.write(struct.pack("<qqq", X.shape[0], X.shape[1], len(off)))
        f.write(off.tobytes() + X.tobytes() + y.tobytes())
    args = [driver, str(data), str(out), str(int(replacement)), repr(float(ratio)), str(int(seed)),
            str(lb), str(le), repr(float(sub_ratio)), str(int(bug_compat)), str(depth), str(bins),
            str(min_inst), str(impurity), repr(float(min_gain)), str(int(tree_seed)), str(agg)]
    p = subprocess.run(args, capture_output=True, text=True, timeout=300,
                       env=None if env is None else dict(os.environ, **env))
    raw = open(out, "rb").read() if os.path.exists(out) else b""
    status = struct.unpack_from("<i", raw, 0)[0] if raw else None
    if status != 0:
        return p, status, None, None, None
    pos = 4
    T = struct.unpack_from("<i", raw, pos)[0]
    pos += 4
    trees, subs = [], []
    for _ in range(T):
        nn, sl = struct.unpack_from("<ii", raw, pos)
        pos += 8
        trees.append(np.frombuffer(raw, np.float64, nn * 8, pos).reshape(nn, 8))
        pos += nn * 64
        subs.append(np.frombuffer(raw, np.int32, sl, pos))
        pos += 4 * sl
    pred = np.frombuffer(raw, np.float64, X.shape[0], pos)
    return p, 0, trees, subs, pred


GBM_DRIVER = os.path.join(ROOT, "tests", "c", "gbm_driver")


def run_gbm_driver(tmp_path, X, y, subspaces, *, L, lr, replacement, ratio, seed, depth, bins,
                   tree_seed):
    """tests/c/gbm_driver: GBMRegressor's loop in C over the shim core (squared loss)."""
    X = np.ascontiguousarray(X, np.float64)
    y = np.ascontiguousarray(y, np.float64)
    data, subs, out = tmp_path / "gdata.bin", tmp_path / "gsubs.bin", tmp_path / "gout.bin"
    with open(data, "wb") as f:
        f.write(struct.pack("<qq", X.shape[0], X.shape[1]) + X.tobytes() + y.tobytes())
    with open(subs, "wb") as f:
        for s in subspaces:
            s = np.asarray(s, np.int32)
            f.write(struct.pack("<i", len(s)) + s.tobytes())
    args = [GBM_DRIVER, str(data), str(subs), str(out), str(L), repr(float(lr)),
            str(int(replacement)), repr(float(ratio)), str(int(seed)), str(depth), str(bins),
            str(int(tree_seed))]
    p = subprocess.run(args, capture_output=True, text=True, timeout=300)
    raw = open(out, "rb").read() if os.path.exists(out) else b""
    status = struct.unpack_from("<i", raw, 0)[0] if raw else None
    if status != 0:
        return p, status, None, None
    pos, trees = 4, []
    for _ in range(L):
        nn = struct.unpack_from("<i", raw, pos)[0]
        pos += 4
        trees.append(np.frombuffer(raw, np.float64, nn * 8, pos).reshape(nn, 8))
        pos += nn * 64
    return p, 0, trees, np.frombuffer(raw, np.float64, X.shape[0], pos)


THREADS = os.path.join(ROOT, "tests", "c", "abi_threads")
THREADS_ASAN = os.path.join(ROOT, "tests", "c", "abi_threads_asan")


def run_threads(tmp_path, X, y, offsets, *, seed, depth, bins, impurity, agg, driver=THREADS,
                env=None, modes=None):
    """tests/c/abi_threads: four jobs fitted + predicted from pthreads (one shared context,
    then four contexts, then with an induced SBAG_EINVAL), each compared byte for byte with
    the serial run inside the driver.  Returns the CompletedProcess."""
    X = np.ascontiguousarray(X, np.float64)
    y = np.ascontiguousarray(y, np.float64)
    off = np.asarray(offsets, np.int64)
    data = tmp_path / "tdata.bin"
    with open(data, "wb") as f:
        f.write(struct.pack("<qqq", X.shape[0], X.shape[1], len(off)))
        f.write(off.tobytes() + X.tobytes() + y.tobytes())
    args = [driver, str(data), str(int(seed)), str(depth), str(bins), str(impurity), str(agg)]
    if modes:
        args.append(modes)
    return subprocess.run(args, capture_output=True, text=True, timeout=600,
                          env=None if env is None else dict(os.environ, **env))
