"""CPU: the plain-C driver of the JNI shim's core builds, links libsbag, and maps a
failing status to the exception class the JNI shim throws (no GPU here: ctxCreate
fails, and the driver reports it instead of crashing)."""
import os
import subprocess

import numpy as np
import pytest

from c_abi_util import DRIVER, GBM_DRIVER, run_driver


@pytest.mark.parametrize("driver", [DRIVER, GBM_DRIVER])
def test_driver_is_built_and_links_libsbag(driver):
    assert os.path.exists(driver), "run __graft_entry__.build()"
    out = subprocess.run(["ldd", driver], capture_output=True, text=True).stdout
    assert "libsbag.so" in out and "not found" not in out


def test_driver_reports_status_as_exception_class(tmp_path):
    import torch

    if torch.cuda.is_available():
        pytest.skip("covered on the GPU by tests/test_gpu_c_abi.py")
    X = np.zeros((4, 2))
    p, status, *_ = run_driver(tmp_path, X, np.zeros(4), [0, 4], replacement=1, ratio=1.0,
                               seed=1, lb=0, le=1, sub_ratio=1.0, bug_compat=1, depth=2, bins=4,
                               min_inst=1, impurity=0, min_gain=0.0, tree_seed=5, agg=0)
    assert p.returncode == 3 and status != 0
    assert "ctxCreate" in p.stdout and "Exception" in p.stdout
