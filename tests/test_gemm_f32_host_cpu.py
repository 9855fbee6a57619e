"""Host-side checks of the fp32 GEMM (ops/csrc/gemm_f32.hip), CPU-only:

- the split-K cost model (dtd_gemm_f32_tn_splits) fills the last round of one-wave-per-SIMD
  workgroups on the BERT-base weight-gradient shapes (f32_num_cus falls back to 256 CUs without
  a GPU);
- ISA audit of the register-direct kernels: inside the main loop no scratch access, and every
  vmcnt wait leaves the next K-step's 14+ loads in flight -- the compiler once sank the one-step
  prefetch down to its use (a vmcnt(0) before the MFMAs), which a straight-line loop body plus
  sched_barriers prevent (profiles/r5_s49_f32_gemm.jsonl)."""
import math
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "distributed_training_and_deepspeed_amd", "ops", "csrc", "gemm_f32.hip")
HIPCC = "/opt/rocm/bin/hipcc" if os.path.exists("/opt/rocm/bin/hipcc") else shutil.which("hipcc")


def _lib_or_skip():
    try:
        from distributed_training_and_deepspeed_amd.ops import _lib
        lib = _lib.lib()
    except Exception as e:  # noqa: BLE001 -- the kernel library is not built here
        pytest.skip(f"kernel library not loadable: {e}")
    if not hasattr(lib, "dtd_gemm_f32_tn_splits"):
        pytest.skip("kernel library predates the fp32 split model")
    return lib


@pytest.mark.parametrize("T", [16384, 32768, 131072])
@pytest.mark.parametrize("o,i", [(2304, 768), (768, 768), (3072, 768), (768, 3072)])
def test_tn_split_model_fills_rounds(T, o, i):
    lib = _lib_or_skip()
    sp = lib.dtd_gemm_f32_tn_splits(o, i, T)
    assert 1 <= sp <= 64
    wgs = (o // 128) * (i // 128) * sp
    slots = 4 * 256                                   # one 128 x 128 wave per SIMD, 256 CUs
    assert wgs / (math.ceil(wgs / slots) * slots) >= 0.9, (o, i, T, sp)


def _function_bodies(asm: str, needle: str):
    bodies, cur, name = {}, None, None
    for line in asm.splitlines():
        m = re.match(r"^(_Z\S+):", line)
        if m:
            name, cur = m.group(1), []
            continue
        if cur is not None:
            if line.strip().startswith("s_endpgm"):
                if needle in name:
                    bodies[name] = cur
                cur = None
                continue
            cur.append(line)
    return bodies


@pytest.mark.skipif(HIPCC is None, reason="hipcc not available")
def test_register_kernels_keep_the_prefetch_in_flight(tmp_path):
    out = tmp_path / "gemm_f32.s"
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-I", os.path.dirname(SRC),
                    "--cuda-device-only", "-S", "-o", str(out), SRC], check=True, capture_output=True)
    # every form: NT x 2 tile widths, NN x 2, TN.  (The NN form with 128 x 96 tiles once waited down
    # to vmcnt(2) right after issuing its next buffer: its dwordx3 [k][n] loads landed in a
    # temporary and were copied into 3-float slots; 4-float vector slots fixed it.)
    bodies = _function_bodies(out.read_text(), "gemm_f32_reg_kernel")
    assert len(bodies) >= 5, sorted(bodies)
    for name, lines in bodies.items():
        start = next(k for k, l in enumerate(lines) if "Inner Loop Header" in l)
        end = next(k for k in range(start + 1, len(lines)) if re.search(r"s_cbranch_\w+ \.LBB", lines[k]))
        loop = lines[start:end + 1]
        assert not any("scratch_" in l for l in loop), name
        assert not any(re.match(r"\s+v_mov_b32", l) for l in loop), name   # no operand copies
        waits = [int(m.group(1)) for l in loop for m in [re.search(r"s_waitcnt vmcnt\((\d+)\)", l)] if m]
        assert waits and min(waits) >= 14, (name, waits)
        assert sum("v_mfma" in l for l in loop) >= 128, name   # both K-steps of the pair
