#!/usr/bin/env python
"""Which RCCL collective breaks hipGraph capture at world 1?  Each case runs in its own child
process (a crash in hipStreamEndCapture kills only that child): capture the collective on a side
stream joined to the capturing stream, replay, compare.  Prints one JSON line per case."""
import json
import os
import subprocess
import sys

CASES = ["all_reduce", "reduce_scatter_tensor", "all_gather_into_tensor", "all_gather_coalesced", "reduce_scatter_coalesced",
         "all_gather_inplace", "reduce_scatter_inplace", "all_reduce_async_wait", "reduce_scatter_async_wait",
         "side_stream_rs", "autograd_rs", "autograd_side_stream_rs", "side_stream_rs_keepwork", "side_stream_rs_evcache",
         "side_stream_rs_join_origin", "side_stream_rs_origin_only", "origin_deferred_wait"]


def child(case):
    import torch
    import torch.distributed as dist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    x = torch.randn(1 << 20, device="cuda", dtype=torch.bfloat16)
    out = torch.empty_like(x)
    xs = [torch.randn(1 << 18, device="cuda", dtype=torch.bfloat16) for _ in range(3)]
    outs = [torch.empty_like(t) for t in xs]

    kept = []

    def side_rs():
        s2 = side[0]
        s2.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s2):
            w = dist.reduce_scatter_tensor(out, x, op=dist.ReduceOp.AVG, async_op=True)
            if case != "side_stream_rs_origin_only":
                w.wait()
            if case == "side_stream_rs_keepwork":
                # the Work object (and the HIP events ProcessGroupNCCL recorded for it) outlives the
                # capture: no hipEventDestroy of a captured event before hipStreamEndCapture
                kept.append(w)
        torch.cuda.current_stream().wait_stream(s2)
        if case in ("side_stream_rs_join_origin", "side_stream_rs_origin_only"):
            # RCCL's internal stream forked from s2: join it into the ORIGIN (capturing) stream
            # directly -- the Work's end event waited on the origin stream
            w.wait()
        del w

    class Hook(torch.autograd.Function):      # issues the collective from the autograd thread
        @staticmethod
        def forward(ctx, t):
            return t * 2

        @staticmethod
        def backward(ctx, g):
            if case == "autograd_side_stream_rs":
                side_rs()
            else:
                dist.reduce_scatter_tensor(out, x, op=dist.ReduceOp.AVG, async_op=True).wait()
            return g * 2
    side = [torch.cuda.Stream()]
    leaf = torch.randn(4096, device="cuda", requires_grad=True)

    def run():
        if case.startswith("side_stream_rs"):
            side_rs()
        elif case in ("autograd_rs", "autograd_side_stream_rs"):
            Hook.apply(leaf).sum().backward()
        elif case == "origin_deferred_wait":
            # issued on the capturing stream, waited only after unrelated work on that stream: in the
            # graph the collective is a branch parallel to that work (ZeRO's captured-step form)
            w = dist.reduce_scatter_tensor(out, x, op=dist.ReduceOp.AVG, async_op=True)
            for _ in range(4):
                leaf.data.mul_(1.0001)
            w.wait()
            out.add_(1.0)
        elif case == "all_reduce":
            dist.all_reduce(x, op=dist.ReduceOp.AVG)
        elif case == "reduce_scatter_tensor":
            dist.reduce_scatter_tensor(out, x, op=dist.ReduceOp.AVG)
        elif case == "all_gather_into_tensor":
            dist.all_gather_into_tensor(out, x)
        elif case == "all_gather_coalesced":
            with dist._coalescing_manager(async_ops=True) as cm:
                for o, i in zip(outs, xs):
                    dist.all_gather_into_tensor(o, i, async_op=True)
            cm.wait()
        elif case == "all_gather_inplace":          # world 1: the shard IS the output
            dist.all_gather_into_tensor(x, x)
        elif case == "reduce_scatter_inplace":
            dist.reduce_scatter_tensor(x, x, op=dist.ReduceOp.AVG)
        elif case == "all_reduce_async_wait":
            dist.all_reduce(x, op=dist.ReduceOp.AVG, async_op=True).wait()
        elif case == "reduce_scatter_async_wait":
            dist.reduce_scatter_tensor(out, x, op=dist.ReduceOp.AVG, async_op=True).wait()
        elif case == "reduce_scatter_coalesced":
            with dist._coalescing_manager(async_ops=True) as cm:
                for o, i in zip(outs, xs):
                    dist.reduce_scatter_tensor(o, i, op=dist.ReduceOp.AVG, async_op=True)
            cm.wait()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        run()                                   # eager warm-up (communicator, buffers)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        run()
    kept.clear()
    if case == "origin_deferred_wait":
        out.zero_()
        g.replay()
        torch.cuda.synchronize()
        want = x.float() + 1.0          # world 1: the reduce-scatter output is the input
        if not torch.allclose(out.float(), want, atol=5e-2):
            print(json.dumps({"case": case, "mismatch": (out.float() - want).abs().max().item()}), flush=True)
            sys.exit(1)
    g.replay()
    torch.cuda.synchronize()
    print(json.dumps({"case": case, "captured_and_replayed": True}), flush=True)
    dist.destroy_process_group()


def main():
    if len(sys.argv) > 2 and sys.argv[1] == "--child":
        child(sys.argv[2])
        return
    for i, case in enumerate(sys.argv[1:] or CASES):
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(29600 + i))
        if case == "side_stream_rs_evcache":
            env["TORCH_NCCL_CUDA_EVENT_CACHE"] = "1"   # events returned to a cache, not destroyed
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", case], env=env,
                           capture_output=True, text=True, timeout=120)
        ok = r.returncode == 0 and "captured_and_replayed" in r.stdout
        print(json.dumps({"case": case, "ok": ok, "returncode": r.returncode,
                          "err": "" if ok else r.stderr.strip().splitlines()[-1][:200] if r.stderr.strip() else ""}), flush=True)
        if r.returncode < 0 or r.returncode >= 128:   # a crashed child: start nothing more on the GPU
            print(json.dumps({"stopped_after": r.returncode}), flush=True)
            sys.exit(3)


if __name__ == "__main__":
    main()
