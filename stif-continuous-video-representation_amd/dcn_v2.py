"""The reference DCNv2 plugin API (codes/models/modules/DCNv2/dcn_v2.py) on the gfx950 op.

``dcn_v2_forward`` is the drop-in for the reference's native ``_ext.dcn_v2_forward``
(vision.cpp:4, dcn_v2.h:9-23); the classes keep the reference's constructor
arguments, parameter names and forward semantics (dcn_v2.py:15-140) so existing
checkpoints load unchanged.  Inference only: backward raises (the reference's
dcn_v2_cuda_backward is out of scope).
"""
from __future__ import annotations

import math

import torch
from torch import nn
from torch.autograd import Function
from torch.nn.modules.utils import _pair

from .ops import dcn_v2_forward  # noqa: F401  (the `_ext` entry point)


class _DCNv2(Function):
    @staticmethod
    def forward(ctx, input, offset, mask, weight, bias, stride, padding, dilation, deformable_groups):
        stride, padding, dilation = _pair(stride), _pair(padding), _pair(dilation)
        kernel_size = _pair(weight.shape[2:4])
        return dcn_v2_forward(input, weight, bias, offset, mask, kernel_size[0], kernel_size[1], stride[0],
                              stride[1], padding[0], padding[1], dilation[0], dilation[1], deformable_groups)

    @staticmethod
    def backward(ctx, grad_output):
        raise NotImplementedError("DCNv2 backward is not implemented (inference engine)")


dcn_v2_conv = _DCNv2.apply


class DCNv2(nn.Module):
    """dcn_v2.py:53-80: weight/bias parameters, offset and mask supplied by the caller."""

    def __init__(self, in_channels, out_channels, kernel_size, stride, padding, dilation=1, deformable_groups=1):
        super().__init__()
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.kernel_size = _pair(kernel_size)
        self.stride = _pair(stride)
        self.padding = _pair(padding)
        self.dilation = _pair(dilation)
        self.deformable_groups = deformable_groups
        self.weight = nn.Parameter(torch.Tensor(out_channels, in_channels, *self.kernel_size))
        self.bias = nn.Parameter(torch.Tensor(out_channels))
        self.reset_parameters()

    def reset_parameters(self):
        n = self.in_channels
        for k in self.kernel_size:
            n *= k
        stdv = 1. / math.sqrt(n)
        self.weight.data.uniform_(-stdv, stdv)
        self.bias.data.zero_()

    def forward(self, input, offset, mask):
        assert 2 * self.deformable_groups * self.kernel_size[0] * self.kernel_size[1] == offset.shape[1]
        assert self.deformable_groups * self.kernel_size[0] * self.kernel_size[1] == mask.shape[1]
        return dcn_v2_conv(input, offset, mask, self.weight, self.bias, self.stride, self.padding,
                           self.dilation, self.deformable_groups)


class DCN(DCNv2):
    """dcn_v2.py:83-107: offsets/mask predicted from the input itself."""

    def __init__(self, in_channels, out_channels, kernel_size, stride, padding, dilation=1, deformable_groups=1):
        super().__init__(in_channels, out_channels, kernel_size, stride, padding, dilation, deformable_groups)
        channels_ = self.deformable_groups * 3 * self.kernel_size[0] * self.kernel_size[1]
        self.conv_offset_mask = nn.Conv2d(self.in_channels, channels_, kernel_size=self.kernel_size,
                                          stride=self.stride, padding=self.padding, bias=True)
        self.init_offset()

    def init_offset(self):
        self.conv_offset_mask.weight.data.zero_()
        self.conv_offset_mask.bias.data.zero_()

    def forward(self, input):
        out = self.conv_offset_mask(input)
        o1, o2, mask = torch.chunk(out, 3, dim=1)
        offset = torch.cat((o1, o2), dim=1)
        mask = torch.sigmoid(mask)
        return dcn_v2_conv(input, offset, mask, self.weight, self.bias, self.stride, self.padding,
                           self.dilation, self.deformable_groups)


class DCN_sep(DCN):
    """dcn_v2.py:110-140: offsets/mask predicted from a separate feature map `fea`."""

    def forward(self, input, fea):
        out = self.conv_offset_mask(fea)
        o1, o2, mask = torch.chunk(out, 3, dim=1)
        offset = torch.cat((o1, o2), dim=1)
        mask = torch.sigmoid(mask)
        return dcn_v2_conv(input, offset, mask, self.weight, self.bias, self.stride, self.padding,
                           self.dilation, self.deformable_groups)
