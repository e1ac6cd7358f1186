"""Reduce the FETCH_SIZE / WRITE_SIZE passes of tools/pmc_kop.sh to bytes per batched K matvec.

The run performs `nops = steps + warmup` batched K matvecs (argv[3], default 13); each op
launches every pass kernel once per RHS chunk (two chunks on two streams at C2), so per
kernel we take the median dispatch value times dispatches / nops, sum over the op's kernels
(setup kernels are excluded by name) and apply the gfx950 FETCH_SIZE correction
(x2, MI355X_MICROARCH.md §HBM)."""
import collections
import csv
import glob
import json
import os
import statistics
import sys

root, out = sys.argv[1], sys.argv[2]
nops = int(sys.argv[3]) if len(sys.argv) > 3 else 13
OP_KERNELS = ("k_row_fwd_t", "k_row_inv_t", "k_pass<float")
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    with open(f) as fh:
        for row in csv.DictReader(fh):
            name = row.get("Kernel_Name", "")
            if any(k in name for k in OP_KERNELS):
                vals[row["Counter_Name"]][name.split("(")[0]].append(float(row["Counter_Value"]))
per = {}
for cnt, ks in vals.items():
    per[cnt] = {k: statistics.median(v) * len(v) / nops for k, v in ks.items()}
fetch_kb = sum(per.get("FETCH_SIZE", {}).values())
write_kb = sum(per.get("WRITE_SIZE", {}).values())
res = {"workload": "C2 batched K matvec, 2-D 1024x1024, 32 RHS, fp32", "M": 1024 * 1024, "rhs": 32,
       "per_kernel_kb": per, "fetch_kb_raw": fetch_kb, "write_kb": write_kb,
       "traffic_bytes_per_op": (2 * fetch_kb + write_kb) * 1024,
       "correction": "FETCH_SIZE x2 (gfx950 counts half of wide streaming reads); units KiB"}
with open(out, "w") as fh:
    json.dump(res, fh, indent=1)
print(json.dumps(res, indent=1))
