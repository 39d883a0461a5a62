"""CPU: the C-ABI library loads, exports every symbol include/sbag.h declares, and
its host-only entry points behave (no compute calls that need a GPU)."""
import ctypes
import os
import re
import shutil

import numpy as np
import pytest

import oracle
from conftest import ROOT

import spark_bagging_amd as sb
from spark_bagging_amd import _native as nat


def declared_symbols():
    txt = open(os.path.join(ROOT, "include", "sbag.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(sbag_\w+)\s*\(", txt, re.M)))


def test_header_declares_expected_entry_points():
    syms = declared_symbols()
    assert set(syms) == set(nat.EXPORTED)


def test_library_exports_every_declared_symbol():
    lib = nat.lib()
    for s in declared_symbols():
        assert hasattr(lib, s), s


def test_library_links_only_hip_runtime():
    """libsbag is a plain C-ABI .so: no torch / python symbols in its dependencies."""
    import subprocess

    out = subprocess.run(["ldd", nat.LIB_PATH], capture_output=True, text=True).stdout
    assert "amdhip64" in out
    assert "torch" not in out and "python" not in out


def test_version_and_error_string():
    lib = nat.lib()
    assert lib.sbag_version().decode().startswith("sbag")
    h = ctypes.c_void_p()
    rc = lib.sbag_ctx_create(9999, ctypes.byref(h))
    assert rc in (nat.SBAG_EINVAL, nat.SBAG_EDEVICE)
    assert len(lib.sbag_last_error()) > 0


@pytest.mark.parametrize("seed", [-1395689524, 42087812, 0, 2**40 + 1])
@pytest.mark.parametrize("ratio", [1.0, 0.7, 0.3])
def test_host_subspace_matches_oracle(seed, ratio):
    assert list(nat.subspace(ratio, 30, seed)) == list(oracle.subspace(ratio, 30, seed))


def test_host_subspace_spark2_anchor():
    """sbag_subspace (host code, no GPU) follows Spark 2.4.3's 64-byte hashSeed:
    XORShiftRandom(0).nextDouble() = 0.8446490682263027, so mkSubspace(u, 1, 0) is []."""
    u = 0.8446490682263027
    assert list(nat.subspace(u, 1, 0)) == []
    assert list(nat.subspace(float(np.nextafter(u, 1.0)), 1, 0)) == [0]


def test_null_arguments_are_rejected():
    lib = nat.lib()
    assert lib.sbag_subspace(1.0, 4, 0, None, None) == nat.SBAG_EINVAL
    assert lib.sbag_fit(None, None, None, None) == nat.SBAG_EINVAL
    assert lib.sbag_fit_booster(None, None, None, None, None) == nat.SBAG_EINVAL
    assert lib.sbag_forest_num_trees(None, None) == nat.SBAG_EINVAL


def test_forest_create_roundtrip_on_host():
    """sbag_forest_create / accessors are host-only: rebuild a forest from node arrays."""
    X, y = sb.load_libsvm(os.path.join(ROOT, "tests", "golden", "data", "vehicle.svm"))
    counts = oracle.bag(True, 0.7, 0, 3, 42087812, [0, 846], 846)
    subs = [oracle.subspace(0.7, 18, 42087812 + i) for i in range(3)]
    f = oracle.fit(X, y, counts, subs, max_depth=4, classification=True)
    trees = [f.tree(t)[0].astype(nat.NODE_DTYPE) for t in range(3)]
    nf = nat.NativeForest.from_trees(trees, subs, nat.IMPURITY_GINI)
    assert len(nf) == 3
    for t in range(3):
        nodes, _ = nf.tree(t)
        assert (nodes == trees[t]).all()
        assert list(nf.subspace(t)) == list(subs[t])


def test_forest_create_rejects_malformed():
    n = np.zeros(1, nat.NODE_DTYPE)
    n["left"], n["right"], n["feature"] = 5, 6, 0
    with pytest.raises(sb.IllegalArgumentException):
        nat.NativeForest.from_trees([n], [[0]], nat.IMPURITY_VARIANCE)


def _leaf(pred):
    n = np.zeros(1, nat.NODE_DTYPE)
    n["left"] = n["right"] = n["feature"] = -1
    n["prediction"] = pred
    return n


def _stump(left, right, feature=0, nn=3):
    n = np.zeros(nn, nat.NODE_DTYPE)
    n["id"] = np.arange(nn)
    n["left"] = n["right"] = n["feature"] = -1
    n[0]["left"], n[0]["right"], n[0]["feature"] = left, right, feature
    n[0]["threshold"] = 0.5
    return n


@pytest.mark.parametrize("case", ["child_back_to_root", "self_loop", "one_child", "right_negative",
                                  "past_end", "feature_out_of_subspace", "same_children"])
def test_forest_create_rejects_bad_links(case):
    """links must point forward inside the tree (pre-order), so a loaded model
    can never make the device walk loop or leave its tree."""
    nodes, sub = {
        "child_back_to_root": (_stump(1, 0), [0]),
        "self_loop": (_stump(0, 2), [0]),
        "one_child": (_stump(1, -1), [0]),
        "right_negative": (_stump(-1, 2), [0]),
        "past_end": (_stump(1, 3), [0]),
        "feature_out_of_subspace": (_stump(1, 2, feature=1), [0]),
        "same_children": (_stump(1, 1), [0]),
    }[case]
    with pytest.raises(sb.IllegalArgumentException):
        nat.NativeForest.from_trees([nodes], [sub], nat.IMPURITY_VARIANCE)


def test_forest_create_rejects_bad_subspace_and_class_ids():
    with pytest.raises(sb.IllegalArgumentException):  # negative global feature index
        nat.NativeForest.from_trees([_stump(1, 2)], [[-3]], nat.IMPURITY_VARIANCE)
    for bad in (-1.0, 2.5, 4096.0, float("nan")):  # a gini leaf must name a class id
        with pytest.raises(sb.IllegalArgumentException):
            nat.NativeForest.from_trees([_leaf(bad)], [[0]], nat.IMPURITY_GINI)
    ok = nat.NativeForest.from_trees([_leaf(4095.0), _stump(1, 2)], [[0], [2]], nat.IMPURITY_GINI)
    assert len(ok) == 2
    # variance leaves may predict anything
    assert len(nat.NativeForest.from_trees([_leaf(-2.5)], [[0]], nat.IMPURITY_VARIANCE)) == 1


def test_loading_a_malformed_model_directory_fails_cleanly(tmp_path):
    """A model directory whose tree data links a child back to its parent loads as Python
    objects but is refused before any kernel sees it."""
    from spark_bagging_amd import persistence as sp

    trees = [_stump(1, 2), _leaf(1.0)]
    model = sb.BaggingRegressionModel([[0], [0]], [sb.DecisionTreeModel(t, np.zeros((len(t), 3)),
                                                                        nat.IMPURITY_VARIANCE)
                                                   for t in trees])
    model.set("numBaseLearners", 2)  # the regression reader counts numBaseLearners (H14)
    path = str(tmp_path / "m")
    model.save(path)
    nodes, stats = sp.read_tree_data(os.path.join(path, "model-0"))
    nodes["right"][0] = 0  # corrupt: right child -> the root
    shutil.rmtree(os.path.join(path, "model-0", "data"))
    sp.write_tree_data(os.path.join(path, "model-0"), nodes, stats)
    back = sb.BaggingRegressionModel.load(path)
    with pytest.raises(sb.IllegalArgumentException):
        back.native_forest()


def test_kernel_barriers_wait_for_lds():
    """Every workgroup barrier in the HIP sources goes through block_sync / block_sync_mem
    (sbag_internal.h), which spell out the s_waitcnt: a bare __syncthreads() let a wave
    cross the barrier with an LDS write in flight on gfx950 (k_split_gini, found by
    scripts/fuzz_parity.py)."""
    import glob
    csrc = os.path.join(ROOT, "spark-bagging_amd", "csrc")
    offenders = []
    for path in sorted(glob.glob(os.path.join(csrc, "*.hip"))):
        for n, line in enumerate(open(path), 1):
            if re.search(r"\b__syncthreads\s*\(", line.split("//")[0]):
                offenders.append(f"{os.path.basename(path)}:{n}")
    assert not offenders, offenders
    helpers = open(os.path.join(csrc, "sbag_internal.h")).read()
    assert "__builtin_amdgcn_s_waitcnt(0xC07F);" in helpers
