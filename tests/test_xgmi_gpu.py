"""Native xGMI all-reduce kernel (comm/csrc/xgmi_allreduce.hip) in local mode: n virtual ranks
on one MI355X exercise the element partition, the per-workgroup release/acquire barrier and the
epoch double-buffering; results must equal the fp32 sum (fixed order) bitwise on every rank."""
import pytest
import torch

from distributed_training_and_deepspeed_amd.comm.xgmi import XgmiAllReduce

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("world", [2, 4, 8])
@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_local_allreduce_exact(world, mode, dtype):
    ar = XgmiAllReduce.local(world, max_bytes=4 << 20, blocks=8)
    try:
        for it, numel in enumerate([8 * world * 3, 65536, 1 << 19]):
            torch.manual_seed(it)
            xs = [torch.randn(numel, device="cuda").to(dtype) for _ in range(world)]
            ref = xs[0].float().clone()
            for x in xs[1:]:
                ref += x.float()
            ref = ref.to(dtype)
            bufs = [x.clone() for x in xs]
            ar.all_reduce_local(bufs, mode=mode)
            torch.cuda.synchronize()
            for b in bufs:
                assert torch.equal(b, ref), (world, mode, numel)
        assert not ar.error()
    finally:
        ar.close()


def test_local_allreduce_average_and_many_epochs():
    ar = XgmiAllReduce.local(4, max_bytes=1 << 20, blocks=16)
    try:
        xs = [torch.full((4096,), float(r + 1), device="cuda") for r in range(4)]
        for _ in range(9):                      # odd count: both parities reused several times
            bufs = [x.clone() for x in xs]
            ar.all_reduce_local(bufs, scale=0.25)
        torch.cuda.synchronize()
        assert all(torch.all(b == 2.5) for b in bufs)
        assert not ar.error()
    finally:
        ar.close()


def _ipc_rank(rank, world, port, out):
    import time
    """Real (IPC) mode: `world` processes on the same GPU map each other's staging and signal buffers
    through hipIpcOpenMemHandle, exactly as ranks on different GPUs of a node do."""
    from distributed_training_and_deepspeed_amd import comm
    comm.init(rank=rank, world_size=world, backend="gloo", init_method=f"file://{out}/rdzv")
    torch.cuda.set_device(0)
    ar = XgmiAllReduce(max_bytes=4 << 20, one_shot_max=64 << 10, blocks=8)
    ok = True
    try:
        for dtype in (torch.bfloat16, torch.float32):
            for it, numel in enumerate([8 * world * 3, 16384, 1 << 19]):   # one-shot, one-shot, two-shot
                g = torch.Generator().manual_seed(1000 * it + 7)
                xs = [torch.randn(numel, generator=g).to(dtype) for _ in range(world)]
                ref = xs[0].float().clone()
                for x in xs[1:]:
                    ref += x.float()
                mine = xs[rank].cuda()
                # uneven arrival: ranks reach the barrier at different times (host sleep on odd
                # ranks, a queued GEMM ahead of the kernel on rank 0) -- the spin barrier must
                # wait, not time out or read stale peer data
                if rank % 2:
                    time.sleep(0.02)
                if rank == 0:
                    big = torch.randn(2048, 2048, device="cuda")
                    for _ in range(8):
                        big = big @ big * 1e-3
                ar.all_reduce(mine, average=(it == 1))
                torch.cuda.synchronize()
                want = (ref / world if it == 1 else ref).to(dtype)
                ok &= torch.equal(mine.cpu(), want)
        ok &= not ar.error()
    finally:
        torch.distributed.barrier()
        ar.close()
        torch.distributed.barrier()
    with open(f"{out}/r{rank}", "w") as f:
        f.write("ok" if ok else "bad")
    comm.destroy()


@pytest.mark.parametrize("world", [2, 4])
def test_ipc_mode_processes_share_one_gpu(tmp_path, free_port, world):
    import torch.multiprocessing as mp
    mp.spawn(_ipc_rank, args=(world, free_port, str(tmp_path)), nprocs=world, join=True)
    assert [(tmp_path / f"r{r}").read_text() for r in range(world)] == ["ok"] * world
