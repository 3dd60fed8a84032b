"""TEST INFRASTRUCTURE ONLY — CPU fp32 restatement of the reference generators.

Each class restates the reference's forward in stock torch.nn ops, keeping
the reference's parameter names (so state_dicts load both ways) and module
construction order (so one seed gives the same initial weights):

  EDSRRef    <- src/model/nets/edsr_net.py:8-67
  DUFRef     <- src/model/nets/duf_net.py:9-214  (backbone _DenseLayer16/28/52)
  DRFRef     <- src/model/nets/drf_net.py:8-147
  DRFSISRRef <- src/model/nets/drf_sisr_net.py:8-50
plus the step helpers the trainers wrap around them:
  denormalize <- src/utils.py:1-20
  psnr        <- src/model/metrics.py:20-36
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as Fn

DATASET_STATS = {"acdc": (54.089, 48.084), "dsb15": (51.193, 52.671)}  # utils.py:13-16


def denormalize(imgs: torch.Tensor, dataset: str) -> torch.Tensor:
    """utils.py:1-20: (x*std + mean).round().clamp(0, 255)."""
    mean, std = DATASET_STATS[dataset]
    return (imgs.clone() * std + mean).round().clamp(0, 255)


def psnr(output: torch.Tensor, target: torch.Tensor, max_value: float = 255.0, size_average: bool = True):
    """metrics.py:20-36: 10*log10(max^2 / (mse + 1e-10)), per sample, then mean."""
    dims = list(range(1, output.dim()))
    mse = Fn.mse_loss(output, target, reduction="none").mean(dims)
    val = 10 * torch.log10(max_value ** 2 / (mse + 1e-10))
    return val.mean() if size_average else val


def ssim(output: torch.Tensor, target: torch.Tensor, dim: int = 2, channels: int = 1, size_average: bool = True,
         value_range: float = 255.0) -> torch.Tensor:
    """metrics.py:39-113 restated: depthwise Gaussian window exp(-((x-mu)/(2*sigma))^2)
    (11 taps, sigma 1.5, product over dims, normalised), valid convolution,
    SSIM map, mean (or per-sample mean)."""
    c1, c2 = (0.01 * value_range) ** 2, (0.03 * value_range) ** 2
    conv = Fn.conv2d if dim == 2 else Fn.conv3d
    grids = torch.meshgrid([torch.arange(11, dtype=torch.float32) for _ in range(dim)], indexing="ij")
    kernel = 1
    for g in grids:
        kernel = kernel * (1 / (1.5 * math.sqrt(2 * math.pi)) * torch.exp(-((g - 5) / (2 * 1.5)) ** 2))
    kernel = (kernel / torch.sum(kernel)).view(1, 1, *kernel.shape).repeat(channels, *[1] * (dim + 1))
    kernel = kernel.to(output.dtype)
    mu1 = conv(output, weight=kernel, groups=channels)
    mu2 = conv(target, weight=kernel, groups=channels)
    s1 = conv(output * output, weight=kernel, groups=channels) - mu1.pow(2)
    s2 = conv(target * target, weight=kernel, groups=channels) - mu2.pow(2)
    s12 = conv(output * target, weight=kernel, groups=channels) - mu1 * mu2
    m = ((2 * mu1 * mu2 + c1) * (2.0 * s12 + c2)) / ((mu1.pow(2) + mu2.pow(2) + c1) * (s1 + s2 + c2))
    if size_average:
        return m.mean()
    return m.mean(dim=list(range(1, output.dim())))


def _pow2_steps(r: int):
    if (math.log(r, 2) % 1) == 0:
        return [2] * int(math.log(r, 2))
    if r == 3:
        return [3]
    raise NotImplementedError


# ---------------------------------------------------------------- EDSR --
class _EDSRRes(nn.Module):
    def __init__(self, f, scale):
        super().__init__()
        self.body = nn.Sequential()
        for name, mod in (("conv1", nn.Conv2d(f, f, 3, padding=1)), ("relu1", nn.ReLU()),
                          ("conv2", nn.Conv2d(f, f, 3, padding=1))):
            self.body.add_module(name, mod)
        self.res_scale = scale

    def forward(self, x):  # edsr_net.py:50-53
        out = self.body(x).mul(self.res_scale)
        out += x
        return out


class EDSRRef(nn.Module):
    def __init__(self, in_channels, out_channels, num_resblocks, num_features, upscale_factor, res_scale=0.1):
        super().__init__()
        f = num_features
        self.upscale_factor = upscale_factor
        self.head = nn.Sequential(nn.Conv2d(in_channels, f, 3, padding=1))
        self.body = nn.Sequential(*[_EDSRRes(f, res_scale) for _ in range(num_resblocks)])
        self.body.add_module("conv", nn.Conv2d(f, f, 3, padding=1))
        up = nn.Sequential()
        for j, s in enumerate(_pow2_steps(upscale_factor), 1):
            up.add_module(f"conv{j}", nn.Conv2d(f, s * s * f, 3, padding=1))
            up.add_module(f"deconv{j}", nn.PixelShuffle(s))
        self.tail = nn.Sequential(up)
        self.tail.add_module("conv", nn.Conv2d(f, out_channels, 3, padding=1))

    def forward(self, x):  # edsr_net.py:34-38
        h = self.head(x)
        return self.tail(self.body(h) + h)


# ----------------------------------------------------------------- DUF --
def _dense_unit(cin, growth, depth_pad):
    """BN3d-ReLU-Conv1x1x1-BN3d-ReLU-Conv3x3x3 (duf_net.py:195-214)."""
    seq = nn.Sequential()
    seq.add_module("bn1", nn.BatchNorm3d(cin))
    seq.add_module("relu1", nn.ReLU())
    seq.add_module("conv1", nn.Conv3d(cin, cin, kernel_size=1))
    seq.add_module("bn2", nn.BatchNorm3d(cin))
    seq.add_module("relu2", nn.ReLU())
    seq.add_module("conv2", nn.Conv3d(cin, growth, kernel_size=3, padding=(depth_pad, 1, 1)))
    return seq


class _DenseStack(nn.Module):
    """_DenseLayer16/28/52 (duf_net.py:102-192): n_keep depth-preserving units,
    3 depth-shrinking units whose concat input is trimmed [:, :, 1:-1]."""

    def __init__(self, f, g, n_keep, tail_in):
        super().__init__()
        self.n_keep = n_keep
        self.n_units = n_keep + 3
        for i in range(self.n_units):
            setattr(self, f"conv{i}", _dense_unit(f, g, 1 if i < n_keep else 0))
            f += g
        self.tail = nn.Sequential()
        self.tail.add_module("bn", nn.BatchNorm3d(tail_in))
        self.tail.add_module("relu", nn.ReLU())
        self.tail.add_module("conv", nn.Conv3d(tail_in, 256, kernel_size=(1, 3, 3), padding=(0, 1, 1)))

    def forward(self, x):
        cat = x
        for i in range(self.n_units):
            y = getattr(self, f"conv{i}")(cat)
            base = cat if i < self.n_keep else cat[:, :, 1:-1]
            cat = torch.cat((base, y), dim=1)
        return self.tail(cat)


_BACKBONES = {"_DenseLayer16": (32, 3, 256), "_DenseLayer28": (16, 9, 256), "_DenseLayer52": (16, 21, 448)}


class DUFRef(nn.Module):
    def __init__(self, in_channels, out_channels, num_frames, size_filter, upscale_factor, backbone):
        super().__init__()
        self.num_frames = num_frames
        self.size_filter = size_filter
        self.upscale_factor = upscale_factor
        g, n_keep, tail_in = _BACKBONES[backbone]
        self.denseLayer = _DenseStack(64, g, n_keep, tail_in)
        self.head = nn.Conv2d(in_channels, 64, kernel_size=3, padding=1)
        k2r2 = size_filter ** 2 * upscale_factor ** 2
        self.filterNet = nn.Sequential()
        for name, mod in (("relu1", nn.ReLU()), ("conv1", nn.Conv3d(256, 512, 1)), ("relu2", nn.ReLU()),
                          ("conv2", nn.Conv3d(512, k2r2, 1))):
            self.filterNet.add_module(name, mod)
        self.residualNet = nn.Sequential()
        for name, mod in (("relu1", nn.ReLU()), ("conv1", nn.Conv3d(256, 256, 1)), ("relu2", nn.ReLU()),
                          ("conv2", nn.Conv3d(256, in_channels * upscale_factor ** 2, 1))):
            self.residualNet.add_module(name, mod)

    def centre(self):
        n = self.num_frames
        return n // 2 if n % 2 == 1 else n // 2 - 1  # duf_net.py:53

    def forward(self, inputs):  # duf_net.py:51-99
        k, r = self.size_filter, self.upscale_factor
        target = inputs[self.centre()].unsqueeze(2)
        feats = torch.stack([self.head(f) for f in inputs], dim=2)
        feats = self.denseLayer(feats)
        filt = self.filterNet(feats)
        filt = filt.reshape(filt.shape[0], k * k, r * r, *filt.shape[2:])
        filt = torch.softmax(filt, dim=1)[:, :, :, 0]  # (N, k*k, r*r, H, W)
        eye = torch.FloatTensor(np.reshape(np.eye(k * k), (k * k, 1, k, k))).to(filt.device, target.dtype)
        outs = []
        for c in range(target.shape[1]):
            patches = Fn.conv2d(target[:, c], eye, padding=k // 2)          # (N, k*k, H, W)
            patches = patches.permute(0, 2, 3, 1).contiguous().unsqueeze(-2)  # (N, H, W, 1, k*k)
            fw = filt.permute(0, 3, 4, 1, 2).contiguous()                   # (N, H, W, k*k, r*r)
            o = torch.matmul(patches, fw).squeeze(-2).permute(0, 3, 1, 2).contiguous()
            outs.append(Fn.pixel_shuffle(o, r))
        out = torch.cat(outs, dim=1)
        res = self.residualNet(feats).squeeze(2)
        return out + Fn.pixel_shuffle(res, r)


# ----------------------------------------------------------------- DRF --
_PROJ = {2: (6, 2, 2), 3: (7, 3, 2), 4: (8, 4, 2), 8: (12, 8, 2)}  # drf_net.py:70-77


def _prelu():
    return nn.PReLU(num_parameters=1, init=0.2)


class _DRFIn(nn.Sequential):  # drf_net.py:52-58
    def __init__(self, cin, f):
        super().__init__()
        self.add_module("conv1", nn.Conv2d(cin, 4 * f, 3, padding=1))
        self.add_module("prelu1", _prelu())
        self.add_module("conv2", nn.Conv2d(4 * f, f, 1))
        self.add_module("prelu2", _prelu())


class _DRFFeedback(nn.Module):  # drf_net.py:61-133
    def __init__(self, f, groups, r):
        super().__init__()
        k, s, p = _PROJ[r]
        self.in_block = nn.Sequential()
        self.in_block.add_module("conv", nn.Conv2d(2 * f, f, 1))
        self.in_block.add_module("prelu", _prelu())
        self.up_blocks = nn.ModuleList()
        self.down_blocks = nn.ModuleList()
        for i in range(groups):
            up, down = nn.Sequential(), nn.Sequential()
            if i == 0:
                up.add_module("deconv", nn.ConvTranspose2d(f, f, k, stride=s, padding=p))
                up.add_module("prelu", _prelu())
                down.add_module("conv", nn.Conv2d(f, f, k, stride=s, padding=p))
                down.add_module("prelu", _prelu())
            else:
                up.add_module("conv1", nn.Conv2d(f * (i + 1), f, 1))
                up.add_module("prelu1", _prelu())
                up.add_module("deconv2", nn.ConvTranspose2d(f, f, k, stride=s, padding=p))
                up.add_module("prelu2", _prelu())
                down.add_module("conv1", nn.Conv2d(f * (i + 1), f, 1))
                down.add_module("prelu1", _prelu())
                down.add_module("conv2", nn.Conv2d(f, f, k, stride=s, padding=p))
                down.add_module("prelu2", _prelu())
            self.up_blocks.append(up)
            self.down_blocks.append(down)
        self.out_block = nn.Sequential()
        self.out_block.add_module("conv", nn.Conv2d(f * groups, f, 1))
        self.out_block.add_module("prelu", _prelu())
        self.hidden_state = None

    def forward(self, x):
        lr = self.in_block(torch.cat([x, self.hidden_state], dim=1))
        lrs, hrs = [lr], []
        for up, down in zip(self.up_blocks, self.down_blocks):
            hrs.append(up(torch.cat(lrs, dim=1)))
            lrs.append(down(torch.cat(hrs, dim=1)))
        return self.out_block(torch.cat(lrs[1:], dim=1))


class _DRFOut(nn.Sequential):  # drf_net.py:136-147
    def __init__(self, f, cout, r):
        super().__init__()
        steps = _pow2_steps(r)
        for j, s in enumerate(steps, 1):
            self.add_module(f"conv{j}", nn.Conv2d(f, s * s * f, 3, padding=1))
            self.add_module(f"pixelshuffle{j}", nn.PixelShuffle(s))
        self.add_module(f"conv{len(steps) + 1}", nn.Conv2d(f, cout, 3, padding=1))


class DRFRef(nn.Module):
    """VSR: list of T frames -> list of T outputs (drf_net.py:38-49)."""

    def __init__(self, in_channels, out_channels, num_features, num_groups, upscale_factor):
        super().__init__()
        if upscale_factor not in _PROJ:
            raise ValueError(f"The upscale factor should be 2, 3, 4 or 8. Got {upscale_factor}.")
        self.in_block = _DRFIn(in_channels, num_features)
        self.f_block = _DRFFeedback(num_features, num_groups, upscale_factor)
        self.out_block = _DRFOut(num_features, out_channels, upscale_factor)

    def step(self, x, first):
        feat = self.in_block(x)
        if first:
            self.f_block.hidden_state = feat
        fb = self.f_block(feat)
        self.f_block.hidden_state = fb
        return self.out_block(feat + fb)

    def forward(self, inputs):
        return [self.step(x, i == 0) for i, x in enumerate(inputs)]


class DRFSISRRef(DRFRef):
    """SISR variant: the same image fed num_steps times (drf_sisr_net.py:39-50)."""

    def __init__(self, in_channels, out_channels, num_steps, num_features, num_groups, upscale_factor):
        super().__init__(in_channels, out_channels, num_features, num_groups, upscale_factor)
        self.num_steps = num_steps

    def forward(self, x):
        return [self.step(x, i == 0) for i in range(self.num_steps)]
