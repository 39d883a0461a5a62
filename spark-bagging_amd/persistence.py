"""Spark 2.4.3 on-disk format of the bagging models.

A GPU-trained forest is written in the directory layout the reference's
MLWriter produces, so stock Spark (with spark-ensemble on the classpath) can load
it, and a model saved by the reference can be loaded here:

  <path>/metadata/part-00000        DefaultParamsWriter.saveMetadata JSON line
                                    (BaggingRegressorParams.saveImpl,
                                    ml/regression/BaggingRegressor.scala:50-66)
  <path>/learner/metadata/...       the base learner (HasBaseLearner.saveImpl,
                                    ml/ensemble/ensembleParams.scala:121-141)
  <path>/model-$i/metadata/...      DecisionTree*Model metadata (+ numFeatures,
                                    numClasses for the classifier)
  <path>/model-$i/data/*.parquet    NodeData rows (Spark's DecisionTreeModelReadWrite)
  <path>/data-$i/part-*.json        {"subspace": [...]}  (BaggingRegressor.scala:285-290)

Readers mirror the reference, including its asymmetry: the
regression reader takes the model count from param numBaseLearners
(BaggingRegressor.scala:305), the classification reader from the metadata field
numBaseModels (BaggingClassifier.scala:307).

Upstream details written from Spark 2.4.3 (not in /root/reference, no JVM here):
DefaultParamsWriter.getMetadataToSave (class, timestamp, sparkVersion, uid,
paramMap, defaultParamMap), NodeData / SplitData, and the parquet row-metadata key
`org.apache.spark.sql.parquet.row.metadata`.  Compatibility with a real Spark
reader is unverified here [verify]; the round trip through this module is tested.
"""
import glob
import json
import os
import time
import uuid

import numpy as np
import pyarrow as pa
import pyarrow.parquet as pq

from . import _native as nat

SPARK_VERSION = "2.4.3"

# Spark 2.4.3 DecisionTree estimator defaults (upstream DecisionTreeParams,
# TreeRegressorParams / TreeClassifierParams, HasSeed = class-name hashCode)
DT_DEFAULTS = {
    "cacheNodeIds": False, "checkpointInterval": 10, "featuresCol": "features", "labelCol": "label",
    "maxBins": 32, "maxDepth": 5, "maxMemoryInMB": 256, "minInfoGain": 0.0,
    "minInstancesPerNode": 1, "predictionCol": "prediction",
}
DTR_DEFAULTS = dict(DT_DEFAULTS, impurity="variance", seed=926680331)
DTC_DEFAULTS = dict(DT_DEFAULTS, impurity="gini", seed=159147643,
                    probabilityCol="probability", rawPredictionCol="rawPrediction")

DTR_CLASS = "org.apache.spark.ml.regression.DecisionTreeRegressor"
DTC_CLASS = "org.apache.spark.ml.classification.DecisionTreeClassifier"
DTR_MODEL_CLASS = "org.apache.spark.ml.regression.DecisionTreeRegressionModel"
DTC_MODEL_CLASS = "org.apache.spark.ml.classification.DecisionTreeClassificationModel"

# NodeData(id, prediction, impurity, impurityStats, gain, leftChild, rightChild, split)
_DARR = pa.list_(pa.field("element", pa.float64(), nullable=False))
NODE_SCHEMA = pa.schema([
    pa.field("id", pa.int32(), nullable=False),
    pa.field("prediction", pa.float64(), nullable=False),
    pa.field("impurity", pa.float64(), nullable=False),
    pa.field("impurityStats", _DARR, nullable=True),
    pa.field("gain", pa.float64(), nullable=False),
    pa.field("leftChild", pa.int32(), nullable=False),
    pa.field("rightChild", pa.int32(), nullable=False),
    pa.field("split", pa.struct([
        pa.field("featureIndex", pa.int32(), nullable=False),
        pa.field("leftCategoriesOrThreshold", _DARR, nullable=True),
        pa.field("numCategories", pa.int32(), nullable=False)]), nullable=True),
])


def _spark_field(name, typ, nullable):
    return {"name": name, "type": typ, "nullable": nullable, "metadata": {}}


_SPARK_DARR = {"type": "array", "elementType": "double", "containsNull": False}
SPARK_ROW_METADATA = json.dumps({"type": "struct", "fields": [
    _spark_field("id", "integer", False), _spark_field("prediction", "double", False),
    _spark_field("impurity", "double", False), _spark_field("impurityStats", _SPARK_DARR, True),
    _spark_field("gain", "double", False), _spark_field("leftChild", "integer", False),
    _spark_field("rightChild", "integer", False),
    _spark_field("split", {"type": "struct", "fields": [
        _spark_field("featureIndex", "integer", False),
        _spark_field("leftCategoriesOrThreshold", _SPARK_DARR, True),
        _spark_field("numCategories", "integer", False)]}, True)]}, separators=(",", ":"))


# ------------------------------------------------------------------ text parts
def _write_part(dirpath, lines, suffix=""):
    """One output partition the way Spark's text/json writers leave it."""
    os.makedirs(dirpath, exist_ok=False)
    name = "part-00000" + (f"-{uuid.uuid4()}-c000{suffix}" if suffix else "")
    with open(os.path.join(dirpath, name), "w") as fh:
        for line in lines:
            fh.write(line + "\n")
    open(os.path.join(dirpath, "_SUCCESS"), "w").close()


def _read_lines(dirpath):
    out = []
    for f in sorted(glob.glob(os.path.join(dirpath, "part-*"))):
        with open(f) as fh:
            out.extend(line for line in fh.read().splitlines() if line.strip())
    return out


def _jsonable(v):
    if isinstance(v, (bool, np.bool_)):
        return bool(v)
    if isinstance(v, (int, np.integer)):
        return int(v)
    if isinstance(v, (float, np.floating)):
        f = float(v)
        if f != f:
            return "NaN"  # DoubleParam.jsonEncode
        if f in (float("inf"), float("-inf")):
            return "Inf" if f > 0 else "-Inf"
        return f
    return v


def save_metadata(path, cls, uid, param_map, default_param_map, extra=None):
    """DefaultParamsWriter.saveMetadata: one compact JSON line in metadata/."""
    meta = {"class": cls, "timestamp": int(time.time() * 1000), "sparkVersion": SPARK_VERSION,
            "uid": uid,
            "paramMap": {k: _jsonable(v) for k, v in param_map.items() if v is not None},
            "defaultParamMap": {k: _jsonable(v) for k, v in default_param_map.items()
                                if v is not None}}
    meta.update(extra or {})
    _write_part(os.path.join(path, "metadata"), [json.dumps(meta, separators=(",", ":"))])


def load_metadata(path, expected_class=None):
    """DefaultParamsReader.loadMetadata, with Spark's class-name check."""
    lines = _read_lines(os.path.join(path, "metadata"))
    if not lines:
        raise nat.IllegalArgumentException(nat.SBAG_EINVAL, f"no metadata under {path}")
    meta = json.loads(lines[0])
    if expected_class is not None and meta["class"] != expected_class:
        raise nat.IllegalArgumentException(
            nat.SBAG_EINVAL, f"Error loading metadata: Expected class name {expected_class} but "
                             f"found class name {meta['class']}")
    return meta


# ------------------------------------------------------------------ tree data
def tree_table(nodes, stats):
    """NodeData rows (pre-order ids, NodeData.build) of one fitted tree."""
    n = len(nodes)
    internal = nodes["left"] >= 0
    feat = np.where(internal, nodes["feature"], -1).astype(np.int32)
    thr = [[float(t)] if i else [] for t, i in zip(nodes["threshold"], internal)]
    split = pa.StructArray.from_arrays(
        [pa.array(feat, pa.int32()), pa.array(thr, _DARR), pa.array(np.full(n, -1, np.int32))],
        fields=list(NODE_SCHEMA.field("split").type))
    cols = [
        pa.array(nodes["id"].astype(np.int32)), pa.array(nodes["prediction"].astype(np.float64)),
        pa.array(nodes["impurity"].astype(np.float64)),
        pa.array([list(map(float, s)) for s in np.asarray(stats, np.float64).reshape(n, -1)], _DARR),
        pa.array(np.where(internal, nodes["gain"], -1.0).astype(np.float64)),
        pa.array(nodes["left"].astype(np.int32)), pa.array(nodes["right"].astype(np.int32)), split]
    meta = {b"org.apache.spark.sql.parquet.row.metadata": SPARK_ROW_METADATA.encode()}
    return pa.Table.from_arrays(cols, schema=NODE_SCHEMA.with_metadata(meta))


def write_tree_data(path, nodes, stats):
    d = os.path.join(path, "data")
    os.makedirs(d, exist_ok=False)
    pq.write_table(tree_table(nodes, stats), os.path.join(d, f"part-00000-{uuid.uuid4()}-c000.snappy.parquet"),
                   compression="snappy")
    open(os.path.join(d, "_SUCCESS"), "w").close()


def read_tree_data(path):
    """DecisionTreeModelReadWrite.loadTreeNodes: NodeData rows sorted by id -> the
    engine's node array (split_bin is not part of Spark's format: -1)."""
    files = sorted(glob.glob(os.path.join(path, "data", "*.parquet")))
    t = pa.concat_tables([pq.read_table(f) for f in files]).to_pydict()
    order = np.argsort(np.asarray(t["id"]), kind="stable")
    n = len(order)
    nodes = np.zeros(n, nat.NODE_DTYPE)
    ids = np.asarray(t["id"], np.int32)[order]
    if not (ids == np.arange(n)).all():
        raise nat.IllegalArgumentException(nat.SBAG_EINVAL, f"{path}: node ids are not 0..{n - 1}")
    nodes["id"] = ids
    nodes["left"] = np.asarray(t["leftChild"], np.int32)[order]
    nodes["right"] = np.asarray(t["rightChild"], np.int32)[order]
    nodes["prediction"] = np.asarray(t["prediction"], np.float64)[order]
    nodes["impurity"] = np.asarray(t["impurity"], np.float64)[order]
    nodes["gain"] = np.asarray(t["gain"], np.float64)[order]
    nodes["split_bin"] = -1
    for k, j in enumerate(order):
        sp = t["split"][j]
        if sp is None or sp["featureIndex"] < 0:
            nodes["feature"][k] = -1
            nodes["threshold"][k] = 0.0
        else:
            if sp["numCategories"] != -1:
                raise nat.IllegalArgumentException(
                    nat.SBAG_EINVAL, f"{path}: categorical splits are not supported")
            nodes["feature"][k] = sp["featureIndex"]
            nodes["threshold"][k] = sp["leftCategoriesOrThreshold"][0]
    width = max((len(s) for s in t["impurityStats"]), default=0)
    stats = np.zeros((n, width), np.float64)
    for k, j in enumerate(order):
        s = t["impurityStats"][j] or []
        stats[k, :len(s)] = s
    return nodes, stats


# ------------------------------------------------------------------ subspaces
def write_subspace(path, subspace):
    _write_part(path, [json.dumps({"subspace": [int(x) for x in subspace]}, separators=(",", ":"))],
                suffix=".json")


def read_subspace(path):
    return [int(x) for x in json.loads(_read_lines(path)[0])["subspace"]]


# ------------------------------------------------------------------ one-row JSON data dirs
def write_json_row(path, row):
    """sparkSession.createDataFrame(Seq(data)).repartition(1).write.json(path): one JSON
    line (GBMRegressionModelWriter's Data(weight, subspace, const), GBMRegressor.scala:551-556)."""
    _write_part(path, [json.dumps(row, separators=(",", ":"))], suffix=".json")


def read_json_row(path):
    return json.loads(_read_lines(path)[0])
