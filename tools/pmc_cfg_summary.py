"""Summarise tools/prof_cfg.sh: per-kernel rocprofv3 stats (from the timing run) and HBM bytes per
batched operator from the FETCH_SIZE / WRITE_SIZE passes (FETCH_SIZE x2: gfx950 counts half of
wide streaming reads, MI355X_MICROARCH.md §HBM), against the SURVEY §8(d) algorithmic bytes of the
profiled operator (argv[5]: K / CINV -> B_K, RT / R -> B_RT, plus the L_R-grid floor of R / R^T,
tools/byte_model.py)."""
import collections
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import byte_model  # noqa: E402

root, nops, shape, rhs = sys.argv[1], int(sys.argv[2]), [int(v) for v in sys.argv[3].split(",")], int(sys.argv[4])
op = sys.argv[5] if len(sys.argv) > 5 else "K"
L_R = [int(v) for v in sys.argv[6].split(",")] if len(sys.argv) > 6 and sys.argv[6] else None
OP_KERNELS = ("k_row_fwd_t", "k_row_inv_t", "k_line_fwd_t", "k_line_inv_t", "k_pass<float")
stats = glob.glob(os.path.join(root, "stats", "**", "*kernel_stats.csv"), recursive=True)
if stats:
    with open(stats[0]) as fh:
        rows = list(csv.DictReader(fh))
    print("kernel stats (timing run):")
    for r in rows[:12]:
        print(f"  {r['Name'][:70]:70s} calls {r['Calls']:>5} avg_us {float(r['AverageNs']) / 1e3:9.1f} pct {float(r['Percentage']):5.1f}")
tot = collections.defaultdict(float)
per = collections.defaultdict(float)     # (kernel, counter) -> KB over the run
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    for f in glob.glob(os.path.join(root, c, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if any(k in row.get("Kernel_Name", "") for k in OP_KERNELS):
                    tot[c] += float(row["Counter_Value"])
                    per[(row["Kernel_Name"][:60], c)] += float(row["Counter_Value"])
bk = byte_model.op_bytes(op, shape)
traffic = (2 * tot["FETCH_SIZE"] + tot["WRITE_SIZE"]) * 1024 / nops
res = {"shape": shape, "rhs": rhs, "op": op, "ops": nops, "fetch_kb_per_op_raw": tot["FETCH_SIZE"] / nops,
       "write_kb_per_op": tot["WRITE_SIZE"] / nops, "traffic_bytes_per_op": traffic,
       "algorithmic_bytes_per_op": rhs * bk, "model": "B_RT" if op in ("RT", "R") else "B_K",
       "traffic_over_algorithmic": traffic / (rhs * bk)}
if op in ("RT", "R") and L_R:
    n = byte_model.ngrid(shape)
    real = all(L >= 2 * v - 1 for L, v in zip(L_R, n))
    fl_rhs, fl_spec = byte_model.floor_rt(shape, L_R, real_spec=real)
    res.update({"L_R": L_R, "real_spectrum": real, "L_R_floor_bytes_per_op_one_chunk": rhs * fl_rhs + fl_spec,
                "traffic_over_L_R_floor": traffic / (rhs * fl_rhs + fl_spec)})
print(json.dumps(res))
for name in sorted({k for k, _ in per}):
    f, w = 2 * per[(name, "FETCH_SIZE")] * 1024 / nops / 1e9, per[(name, "WRITE_SIZE")] * 1024 / nops / 1e9
    print(f"  per op: {name:60s} fetch(x2) {f:8.3f} GB  write {w:8.3f} GB")
