"""Probe torch.mode / torch.median tie rules on the GPU (values and returned indices) along dim 1 of
an NCHW tensor, so the fused channel-statistics kernel can follow the same rule."""
import torch

import sys
dev = torch.device(sys.argv[1] if len(sys.argv) > 1 else "cuda:0")
g = torch.Generator().manual_seed(0)
for C in (8, 86, 129):
    for dt in (torch.bfloat16, torch.float32):
        x = torch.randint(0, 6, (4, C, 16, 16), generator=g).to(dt)
        xg = x.to(dev)
        mv, mi = xg.mode(dim=1)
        dv, di = xg.median(dim=1)
        mv, mi, dv, di = mv.cpu(), mi.cpu(), dv.cpu(), di.cpu()
        xs = x.permute(0, 2, 3, 1).reshape(-1, C).float()
        mv, mi, dv, di = [t.reshape(-1) for t in (mv, mi, dv, di)]
        stats = dict(mode_smallest=0, mode_largest=0, mode_first=0, mode_last=0, mode_other=0,
                     med_first=0, med_last=0, med_other=0, med_stable_rank=0, n=xs.shape[0])
        for r in range(xs.shape[0]):
            row = xs[r]
            vals, counts = row.unique(return_counts=True)
            best = counts.max()
            cands = vals[counts == best]
            stats["mode_smallest"] += int(mv[r].float() == cands.min())
            stats["mode_largest"] += int(mv[r].float() == cands.max())
            pos = (row == mv[r].float()).nonzero().flatten()
            stats["mode_first"] += int(mi[r] == pos[0])
            stats["mode_last"] += int(mi[r] == pos[-1])
            stats["mode_other"] += int(mi[r] != pos[0] and mi[r] != pos[-1])
            pos = (row == dv[r].float()).nonzero().flatten()
            stats["med_first"] += int(di[r] == pos[0])
            stats["med_last"] += int(di[r] == pos[-1])
            stats["med_other"] += int(di[r] != pos[0] and di[r] != pos[-1])
            # stable rank: the element at sorted position (C-1)//2 of a stable sort
            order = torch.sort(row, stable=True).indices
            stats["med_stable_rank"] += int(di[r] == order[(C - 1) // 2])
        print(C, dt, stats)
# all-distinct values
x = torch.randn(64, 86, 4, 4, generator=g)
mv, mi = x.to(dev).mode(dim=1)
print("distinct: mode == min", bool((mv.cpu() == x.min(dim=1).values).all()),
      "idx == argmin", bool((mi.cpu() == x.argmin(dim=1)).all()))
# std dtype / precision: bf16 input
xb = torch.randn(2, 86, 8, 8, generator=g).to(torch.bfloat16)
s = xb.to(dev).std(dim=1)
print("std out dtype", s.dtype, "max |gpu - fp64-rounded| ulp-ish",
      (s.cpu().float() - xb.double().std(dim=1).to(torch.bfloat16).float()).abs().max().item())
