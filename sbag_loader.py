"""Import helper: registers the `spark-bagging_amd/` package as `spark_bagging_amd`."""
import importlib.util
import os
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.join(ROOT, "spark-bagging_amd")


def load():
    if "spark_bagging_amd" in sys.modules:
        return sys.modules["spark_bagging_amd"]
    spec = importlib.util.spec_from_file_location(
        "spark_bagging_amd", os.path.join(PKG_DIR, "__init__.py"),
        submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["spark_bagging_amd"] = mod
    spec.loader.exec_module(mod)
    return mod
