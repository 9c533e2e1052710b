"""Restatement of upstream AdaFace ``net.py`` (IR backbones) — ORACLE, test-only.

The reference does ``import net`` (``face_embedder.py:11``) from its *parent*
directory (``face_embedder.py:3``) and calls ``net.build_model(architecture)``
(``face_embedder.py:49``), then ``load_state_dict`` with the ``model.``-stripped
checkpoint keys (``face_embedder.py:51-53``) and ``features, norm =
self.model(x)`` (``face_embedder.py:119,157``).  ``net.py`` is upstream
mk-minchul/AdaFace and is not vendored; this module restates its published
IR backbone so that the state-dict key layout, the op order and the fp32
numerics are those of the reference path:

    input_layer   = Conv3x3(3,64,s1,p1,nobias) -> BN2d(64) -> PReLU(64)
    body[i]       = BasicBlockIR(in, depth, stride)
        res_layer = BN2d(in) -> Conv3x3(in,depth,s1,p1) -> BN2d(depth) ->
                    PReLU(depth) -> Conv3x3(depth,depth,stride,p1) -> BN2d(depth)
        shortcut  = MaxPool2d(1, stride)             if in == depth
                  = Conv1x1(in,depth,stride) -> BN2d if in != depth
        out       = res + shortcut
    output_layer  = BN2d(512) -> Dropout(0.4) -> Flatten (NCHW .view) ->
                    Linear(512*7*7, 512) -> BN1d(512, affine=False)
    forward tail  = norm = ||x||_2 (dim 1, keepdim); out = x / norm

Units per stage: ir_50 = 3/4/14/3, ir_101 ("100 layers") = 3/13/30/3, widths
64/128/256/512; the first unit of each stage has stride 2.  Parameter counts
(43,585,600 / 65,150,912) and state-dict key counts (468 / 918) match the
survey probe of AdaFace's published model sizes.
"""
from __future__ import annotations

from typing import List, Tuple

import torch
from torch import nn

# units per stage, from upstream get_blocks(num_layers)
STAGE_UNITS = {
    "ir_18": (2, 2, 2, 2),
    "ir_34": (3, 4, 6, 3),
    "ir_50": (3, 4, 14, 3),
    "ir_101": (3, 13, 30, 3),
}
STAGE_WIDTHS = (64, 128, 256, 512)


def block_specs(architecture: str) -> List[Tuple[int, int, int]]:
    """(in_channel, depth, stride) for every BasicBlockIR, upstream get_blocks()."""
    if architecture not in STAGE_UNITS:
        raise ValueError("not a correct model name", architecture)
    specs = []
    in_ch = 64
    for units, depth in zip(STAGE_UNITS[architecture], STAGE_WIDTHS):
        specs.append((in_ch, depth, 2))
        specs.extend((depth, depth, 1) for _ in range(units - 1))
        in_ch = depth
    return specs


class Flatten(nn.Module):
    def forward(self, x):
        return x.view(x.size(0), -1)


class BasicBlockIR(nn.Module):
    def __init__(self, in_channel: int, depth: int, stride: int):
        super().__init__()
        if in_channel == depth:
            self.shortcut_layer = nn.MaxPool2d(1, stride)
        else:
            self.shortcut_layer = nn.Sequential(
                nn.Conv2d(in_channel, depth, (1, 1), stride, bias=False),
                nn.BatchNorm2d(depth))
        self.res_layer = nn.Sequential(
            nn.BatchNorm2d(in_channel),
            nn.Conv2d(in_channel, depth, (3, 3), (1, 1), 1, bias=False),
            nn.BatchNorm2d(depth),
            nn.PReLU(depth),
            nn.Conv2d(depth, depth, (3, 3), stride, 1, bias=False),
            nn.BatchNorm2d(depth))

    def forward(self, x):
        return self.res_layer(x) + self.shortcut_layer(x)


class Backbone(nn.Module):
    def __init__(self, architecture: str):
        super().__init__()
        self.input_layer = nn.Sequential(
            nn.Conv2d(3, 64, (3, 3), 1, 1, bias=False), nn.BatchNorm2d(64), nn.PReLU(64))
        self.output_layer = nn.Sequential(
            nn.BatchNorm2d(512), nn.Dropout(0.4), Flatten(),
            nn.Linear(512 * 7 * 7, 512), nn.BatchNorm1d(512, affine=False))
        self.body = nn.Sequential(*[BasicBlockIR(i, d, s) for i, d, s in block_specs(architecture)])

    def forward(self, x):
        x = self.input_layer(x)
        for module in self.body:
            x = module(x)
        x = self.output_layer(x)
        norm = torch.norm(x, 2, 1, True)
        return torch.div(x, norm), norm


def build_model(architecture: str = "ir_50") -> Backbone:
    """Same entry point and error as upstream ``net.build_model``."""
    if architecture not in ("ir_50", "ir_101", "ir_34", "ir_18"):
        raise ValueError("not a correct model name", architecture)
    return Backbone(architecture)


def load_oracle(architecture: str, state_dict) -> Backbone:
    """Build, load an AdaFace-keyed state dict (no ``model.`` prefix), eval()."""
    m = build_model(architecture)
    m.load_state_dict({k: torch.as_tensor(v) for k, v in state_dict.items()})
    return m.eval()
