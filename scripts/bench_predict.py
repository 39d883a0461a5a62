#!/usr/bin/env python3
"""Transform throughput: one C3 forest (128 depth-8 trees on
10M x 100 synthetic rows), then BaggingRegressionModel.transform over the
device-resident rows (sbag_predict_dataset: slicer + tree walk + in-order mean).
Prints rows/s and rows x trees/s; wall time includes the 80 MB result copy."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import sbag_loader  # noqa: E402

sb = sbag_loader.load()
nat = sb._native
N = int(os.environ.get("ROWS", 10_000_000))
L = int(os.environ.get("LEARNERS", 128))
ctx = nat.Context(0)
ds = nat.DeviceDataset.synthetic(N, 100, seed=20261015, num_classes=0, ctx=ctx)
part = [int(round(i * N / 128)) for i in range(129)]
forest = nat.fit(ctx, ds, replacement=True, sample_ratio=1.0, seed=-1395689524, learner_begin=0,
                 learner_end=L, partition_offsets=part, max_depth=8, max_bins=32)
out = nat.predict_dataset(ctx, forest, ds, nat.AGG_MEAN)  # warm-up (forest upload)
reps = 5
t0 = time.perf_counter()
for _ in range(reps):
    out = nat.predict_dataset(ctx, forest, ds, nat.AGG_MEAN)
dt = (time.perf_counter() - t0) / reps
print(json.dumps({"rows": N, "trees": L, "ms": round(dt * 1e3, 3), "rows_per_s": N / dt,
                  "row_trees_per_s": N * L / dt, "checksum": float(out[:1000].sum())}))
forest.free()
ds.free()
ctx.close()
