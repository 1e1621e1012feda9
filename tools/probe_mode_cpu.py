"""CPU torch.mode on all-distinct channel values: is the mode always the minimum (every count 1)?
Diagnoses the rule the fused channel-statistics kernel must follow on the CPU side."""
import torch

g = torch.Generator().manual_seed(0)
for C in (8, 86, 129):
    for dt in (torch.bfloat16, torch.float32):
        torch.randint(0, 6, (4, C, 16, 16), generator=g)
x = torch.randn(64, 86, 4, 4, generator=g)
mv, mi = x.mode(dim=1)
mn = x.min(dim=1).values
bad = (mv != mn)
print("bad", bad.sum().item())
for i in bad.nonzero()[:3]:
    col = x[i[0], :, i[1], i[2]]
    v, c = col.unique(return_counts=True)
    print(mv[tuple(i)].item(), mn[tuple(i)].item(), c.max().item(), v[c == c.max()])
