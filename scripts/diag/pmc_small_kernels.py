"""Per-dispatch means of duration, shader clock and L2 / HBM traffic for the small memory-bound
kernels of a profiled step (rocprofv3 --pmc GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum
TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum, csv) -- round 4 s40: why they run longer after RCCL init."""
import csv
import json
import re
import sys
from collections import defaultdict

FAM = r"(splitk_reduce_kernel|colsum_finalize_kernel|ln_fwd_wave|ln_bwd_wave|adam_kernel|gemm_bt_persistent<\d+|Cijk\w{0,12}|attn_\w+_kernel)"


def main(path, label):
    per = defaultdict(dict)
    for r in csv.DictReader(open(path)):
        key = (r["Dispatch_Id"], r["Kernel_Name"])
        per[key][r["Counter_Name"]] = float(r["Counter_Value"])
        per[key]["_dur"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    fam = defaultdict(lambda: defaultdict(float))
    for (_, name), c in per.items():
        m = re.search(FAM, name)
        if not m:
            continue
        f = fam[m.group(1)]
        f["n"] += 1
        for k, v in c.items():
            f[k] += v
    out = {}
    for k, f in fam.items():
        n = f["n"]
        out[k] = {"n": int(n), "us": round(f["_dur"] / n * 1e6, 1),
                  "ghz": round(f["GRBM_GUI_ACTIVE"] / 8 / f["_dur"] / 1e9, 3) if f["_dur"] else None,
                  **{c: round(f[c] / n) for c in ("TCC_HIT_sum", "TCC_MISS_sum", "TCC_EA0_RDREQ_sum", "TCC_EA0_WRREQ_sum")}}
    print(json.dumps({"label": label, "families": out}))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
