"""Where does the fused GELU-forward GEMM's activation output differ from act(U)?"""
import sys, os; sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import torch
from distributed_training_and_deepspeed_amd.ops import gemm as G
from distributed_training_and_deepspeed_amd.ops import functional as Fx

for M in (512, 8448):
    torch.manual_seed(1)
    N, K = 3072, 768
    x = torch.randn(M, K, device="cuda").bfloat16()
    w = (torch.randn(N, K, device="cuda") * 0.05).bfloat16()
    b = torch.randn(N, device="cuda").bfloat16()
    u, a = G.linear_gelu(x, w, b, "gelu")
    unf = Fx.act_fwd(u, "gelu")
    bad = (a.float() - unf.float()).abs() > 0.05
    print("M", M, "bad", int(bad.sum()), "of", bad.numel())
    if bad.any():
        r, c = bad.nonzero(as_tuple=True)
        print(" rows%256 hist", torch.bincount(r % 256, minlength=256).nonzero().flatten()[:40].tolist())
        print(" cols%256 hist", torch.bincount(c % 256, minlength=256).nonzero().flatten()[:40].tolist())
        print(" row tiles", torch.unique(r // 256).tolist()[:20], "col tiles", torch.unique(c // 256).tolist()[:20])
        i = 0
        print(" sample a", a[r[i], c[i]].item(), "unf", unf[r[i], c[i]].item(), "u", u[r[i], c[i]].item())
        uref = (x.float() @ w.float().t() + b.float()).bfloat16()
        ub = (u != uref)[bad]
        print(" u differs from uref at bad:", float(ub.float().mean()), " u differs anywhere:", int((u.float() - uref.float()).abs().gt(0.05).sum()))
        for i in range(4):
            print("  a", a[r[i], c[i]].item(), "act(u)", unf[r[i], c[i]].item(), "u", u[r[i], c[i]].item(), "uref", uref[r[i], c[i]].item())
        print(" a==0 frac", float((a[bad] == 0).float().mean()), " a==u frac", float((a[bad] == u[bad]).float().mean()))
