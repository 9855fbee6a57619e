#!/usr/bin/env python
"""Per-kernel-family effective clock and MFMA-pipe utilisation of a profiled training step
(rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA ...).

  effective clock  = GRBM_GUI_ACTIVE / 8 XCDs / dispatch wall time
  MFMA utilisation = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 * 1024 SIMDs)
  (SQ_VALU_MFMA_BUSY_CYCLES = 16 cycles per v_mfma_f32_16x16x32_bf16 / 32 per 32x32x16 summed over
  SIMDs, i.e. 1024 bf16 FLOP per busy cycle: 100 % = the 2.5 PF/s spec at 2.4 GHz.)
Dispatches shorter than 100 us are left out of the clock column (the quotient reads high)."""
import csv
import json
import re
import sys
from collections import defaultdict


def family(name: str) -> str:
    if "Cijk" in name:
        return "hipBLASLt GEMM"
    m = re.search(r"(gemm_bt_persistent<\d+|gemm_w4_kernel<\d+|gemm_f32_kernel<\w+>|wgrad_tn_kernel|gemm_tn\w*|attn_\w+_kernel\w*|ln_\w+_wave|emb_ln_fwd_wave|adam_kernel|xent_\w+_kernel|"
                  r"splitk_reduce_kernel|embed_\w+_kernel|colsum_finalize_kernel|act_\w+_kernel|dropout_kernel)", name)
    return m.group(1) if m else "other"


def main(path, steps, by_name=False):
    per = defaultdict(dict)
    for r in csv.DictReader(open(path)):
        key = (r["Dispatch_Id"], r["Kernel_Name"])
        per[key][r["Counter_Name"]] = float(r["Counter_Value"])
        per[key]["_dur"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    fam = defaultdict(lambda: defaultdict(float))
    for (_, name), c in per.items():
        f = fam[name[:110] if by_name else family(name)]
        f["n"] += 1
        f["dur"] += c["_dur"]
        f["cyc"] += c.get("GRBM_GUI_ACTIVE", 0) / 8
        f["mfma_busy"] += c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0)
        f["mfma"] += c.get("SQ_INSTS_MFMA", 0)
        f["valu"] += c.get("SQ_INSTS_VALU", 0)
        if c["_dur"] >= 1e-4:
            f["dur_long"] += c["_dur"]
            f["cyc_long"] += c.get("GRBM_GUI_ACTIVE", 0) / 8
    rows = []
    for k, f in sorted(fam.items(), key=lambda kv: -kv[1]["dur"]):
        if f["dur"] < 1e-4 * steps:
            continue
        rows.append({"kernel": k, "ms_per_step": round(f["dur"] / steps * 1e3, 3), "n_per_step": round(f["n"] / steps, 1),
                     "eff_clock_GHz": round(f["cyc_long"] / f["dur_long"] / 1e9, 2) if f["dur_long"] else None,
                     "mfma_util": round(f["mfma_busy"] / (f["cyc"] * 1024), 3) if f["cyc"] else None,
                     "bf16_TFs_from_busy": round(f["mfma_busy"] * 1024 / f["dur"] / 1e12, 1) if f["dur"] else None,
                     "valu_per_mfma": round(f["valu"] / f["mfma"], 2) if f["mfma"] else None})
    for r in rows:
        print(json.dumps(r))


if __name__ == "__main__":
    # a third argument "name" groups by kernel name instead of family
    main(sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 1.0, len(sys.argv) > 3 and sys.argv[3] == "name")
