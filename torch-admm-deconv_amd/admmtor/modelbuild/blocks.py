"""Building blocks of the config-5 caller: DivergentAttention and its conv branches.

Module trees, parameter names, registration order and seeded initialisation follow
/root/reference/src/admmtor/modelbuild/blocks.py so reference checkpoints (and
optimizer states) load unchanged:

  DivergentAttention   blocks.py:158-204   convout, convs.{2i} 1x1 conv, convs.{2i+1} UpDownBlock,
                                           attentions.{i} CBAM, admms.{i} ADMMDeconv (the HIP solver)
  UpDownBlock          blocks.py:207-230   chx(x) + chc2(down(chc(up(x))))
  UpBlock / DownBlock  blocks.py:264-313   3x3 transposed conv (H+2) / valid conv (back to H)
  MultiADMM            blocks.py:252-261   concat of several ADMMDeconv outputs
  default_init_weights blocks.py:343-351   xavier-normal weights, zero bias (Conv2d/ConvTranspose2d only)
"""
import torch
import torch.nn as nn
from torch.utils.checkpoint import checkpoint

from admmtor.elayers.admmdeconv import ADMMDeconv
from admmtor.elayers.attentions import CBAM
from admmtor.eops.deconv import fft_admm_tv_grouped


@torch.no_grad()
def default_init_weights(nn_modules):
    """Xavier-normal weights, zero bias, for Conv2d / ConvTranspose2d; anything else is left alone
    (so a container such as UpDownBlock keeps PyTorch's default init, as in the reference)."""
    for m in (nn_modules if isinstance(nn_modules, list) else [nn_modules]):
        if isinstance(m, (nn.Conv2d, nn.ConvTranspose2d)):
            nn.init.xavier_normal_(m.weight)
            if m.bias is not None:
                m.bias.zero_()


class _Stage(nn.Module):
    """conv -> optional normalisation -> optional activation -> optional stride-1 max pool."""

    def _post(self, x):
        for step in (self.normalization, self.activation, self.max_pool):
            if step is not None:
                x = step(x)
        return x


class DownBlock(_Stage):
    def __init__(self, in_channels: int, out_channels: int, kernel_size, activation: nn.Module = None,
                 normalization: nn.Module = None, pool_size: int = 0):
        super().__init__()
        ks = kernel_size if isinstance(kernel_size, tuple) else (kernel_size, kernel_size)
        self.down_conv = nn.Conv2d(in_channels, out_channels, kernel_size=ks, stride=1,
                                   padding=max(0, pool_size - 1), padding_mode="zeros", bias=False)
        default_init_weights(self.down_conv)
        self.normalization = normalization
        self.activation = activation
        self.max_pool = nn.MaxPool2d(kernel_size=pool_size, stride=1) if pool_size else None

    def forward(self, x):
        return self._post(self.down_conv(x))


class UpBlock(_Stage):
    def __init__(self, in_channels: int, out_channels: int, kernel_size, activation: nn.Module = None,
                 normalization: nn.Module = None, pool_size: int = 0):
        super().__init__()
        self.up_conv = nn.ConvTranspose2d(in_channels, out_channels, kernel_size=kernel_size, stride=1, bias=False)
        default_init_weights(self.up_conv)
        self.normalization = normalization
        self.max_pool = nn.MaxPool2d(kernel_size=pool_size, stride=1) if pool_size else None
        self.activation = activation

    def forward(self, x):
        return self._post(self.up_conv(x))


class UpDownBlock(nn.Module):
    def __init__(self, up_in_ch: int, up_out_ch: int, down_out_ch: int, kernel_size,
                 activation: nn.Module = None, normalization: nn.Module = None, pool_size: int = 0):
        super().__init__()
        self.up_block = UpBlock(up_in_ch, up_out_ch, kernel_size, normalization, activation, pool_size)
        self.down_block = DownBlock(up_out_ch, down_out_ch, kernel_size, normalization, activation, pool_size)
        self.chc = nn.Conv2d(up_out_ch, up_out_ch, kernel_size=1, bias=False)
        self.chc2 = nn.Conv2d(down_out_ch, down_out_ch, kernel_size=1, bias=False)
        self.chx = nn.Conv2d(up_in_ch, down_out_ch, kernel_size=1, bias=True)

    def forward(self, x):
        return self.chx(x) + self.chc2(self.down_block(self.chc(self.up_block(x))))


def _branch_plan(n_convs: int, n_attn: int):
    """Which conv outputs meet which attention, following the reference's zip() pairing
    (blocks.py:199-202): the first half of the attentions pairs with the first half of the conv
    outputs, the second half with the second half, each zip truncated to the shorter list.
    Conv outputs that meet no attention do not reach the result, so they are not computed
    (same outputs and gradients as the reference, which computes and drops them)."""
    h_att, h_out = n_attn // 2, n_convs // 2
    first = [(a, a) for a in range(min(h_att, h_out))]
    second = [(h_att + j, h_out + j) for j in range(min(n_attn - h_att, n_convs - h_out))]
    return first, second


class DivergentAttention(nn.Module):
    def __init__(self, branches: int, in_channels: int, out_channels: int, conv_filters: int, gate_channels: int,
                 attention_reduction: int, out_activation: nn.Module = None, admms: list = None):
        super().__init__()
        if admms is not None:
            assert len(admms) == branches
        self._pool_types = [("avg", "max"), ("lp", "lse")]
        self.admms = nn.ModuleList() if admms is not None else None
        self.out_activation = out_activation if out_activation is not None else nn.Identity()
        self.convs = nn.ModuleList()
        self.attentions = nn.ModuleList()
        self.convout = nn.Conv2d(conv_filters * branches, out_channels, kernel_size=1, bias=True)
        for i in range(branches):
            self.convs.append(nn.Conv2d(in_channels, conv_filters, kernel_size=1, bias=True))
            self.convs.append(UpDownBlock(up_in_ch=in_channels, up_out_ch=in_channels, down_out_ch=conv_filters,
                                          kernel_size=3))
            self.attentions.append(CBAM(gate_channels=gate_channels, reduction_ratio=attention_reduction,
                                        pool_types=self._pool_types[i % 2], use_spatial=True))
            if admms is not None:
                self.admms.append(ADMMDeconv(**admms[i]))
        for conv in self.convs:
            default_init_weights(conv)
        default_init_weights(self.convout)
        # recompute each conv+attention branch in the backward instead of keeping its
        # activations (off by default; see set_branch_checkpointing)
        self.checkpoint_branches = False
        # solve ADMM modules that share x together (see _admm_outputs); plain attribute, not state
        self.group_admms = True

    def _admm_outputs(self, x):
        """Every ADMM module applied to x.  Modules that differ only in lambda / rho (no PSF, the
        same iterations and shrink -- train.py's DECONV1/DECONV2) are solved together in one
        native pass sequence (fft_admm_tv_grouped, desc.groups); otherwise one call each."""
        mods = list(self.admms)
        groupable = (self.group_admms and len(mods) > 1 and x.is_cuda and x.dim() == 4
                     and all(m.w.numel() == 0 and m.max_iters == mods[0].max_iters and m.iso == mods[0].iso
                             for m in mods))
        if groupable:
            from admmtor import _native
            groupable = _native.load().admm_tv_supported(x.shape[-2], x.shape[-1]) in (1, 3)
        if not groupable:
            return [m(x) for m in mods]
        sols = fft_admm_tv_grouped(x, [m.lmbda for m in mods], [m.rho for m in mods], mods[0].w,
                                   mods[0].iso, mods[0].max_iters)
        return [m.activation(sol + m.b) for m, sol in zip(mods, sols)]  # ADMMDeconv.forward's tail

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        n_convs = len(self.convs) if self.admms is None else min(len(self.convs), len(self.admms))
        first, second = _branch_plan(n_convs, len(self.attentions))
        restored = self._admm_outputs(x) if self.admms is not None else None

        def branch(a, o, inp):
            f = self.convs[o](inp if restored is None else restored[o])
            return self.attentions[a](f) + f

        def gated(pairs):
            if self.checkpoint_branches and self.admms is None and torch.is_grad_enabled():
                feats = [checkpoint(branch, a, o, x, use_reentrant=False) for a, o in pairs]
            else:
                feats = [branch(a, o, x) for a, o in pairs]
            return torch.cat(feats, dim=1)

        left, right = gated(first), gated(second)
        return self.out_activation(self.convout(torch.cat([left * right, left + right], dim=1)))


def set_branch_checkpointing(model: nn.Module, enabled: bool = True) -> int:
    """Turn branch recomputation on for every DivergentAttention without ADMM modules in `model`
    (the wide levels of DivergentRestorer).  Outputs and gradients are unchanged (the branches are
    deterministic); activation memory drops from O(branches x feature maps) to O(branches) feature
    maps, which is what lets config 5 (batch 16 at 512^2) fit in one GPU's 288 GB.  Returns the
    number of blocks switched."""
    n = 0
    for m in model.modules():
        if isinstance(m, DivergentAttention) and m.admms is None:
            m.checkpoint_branches = enabled
            n += 1
    return n


class MultiADMM(nn.Module):
    """Channel-concatenation of several ADMM restorations of the same input (blocks.py:252-261)."""

    def __init__(self, admm_dicts: list):
        super().__init__()
        self.admms = nn.ModuleList([ADMMDeconv(**d) for d in admm_dicts])

    def forward(self, x):
        return torch.cat([m(x) for m in self.admms], dim=1)
