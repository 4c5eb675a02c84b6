"""Drop-in replacement for the reference ``unet3D`` module (TThuraya/multimodal-PL unet3D.py).

Same class / factory names, constructor signatures, forward signatures, return tuples and state_dict keys
(checkpoints interchange: the fp32 NCDHW parameters ARE the reference parameters). The forward of every
trunk model runs on the MI355X-native executor (u3d.trunk -> libu3d.so HIP kernels); there is no CPU
path: calling a model on CPU tensors raises U3DError.

Precision: fp32 by default (parity mode); under ``torch.autocast('cuda')`` (the reference's --FP16 path)
activations are bf16 with fp32 accumulation and fp32 master weights.
"""
import torch
import torch.nn as nn

from u3d import subgraph, trunk
from u3d._lib import U3DError

affine_par = True
in_place = True


class Conv3d(nn.Conv3d):
    """Weight-standardised Conv3d, reference unet3D.py:16-27."""

    def __init__(self, in_channels, out_channels, kernel_size, stride=(1, 1, 1), padding=(0, 0, 0),
                 dilation=(1, 1, 1), groups=1, bias=False):
        super().__init__(in_channels, out_channels, kernel_size, stride, padding, dilation, groups, bias)

    def forward(self, x):
        return _conv_module_forward(self, x, standardize=True)


def _conv_module_forward(m, x, standardize):
    k, s, p = m.kernel_size[0], m.stride[0], m.padding[0]
    if (m.kernel_size != (k, k, k) or m.stride != (s, s, s) or k not in (1, 3) or s not in (1, 2)
            or m.padding != (k // 2,) * 3 or m.groups != 1 or m.dilation != (1, 1, 1) or m.bias is not None
            or m.in_channels % 8 != 0):
        raise U3DError(f"u3d: Conv3d k={m.kernel_size} s={m.stride} p={m.padding} cin={m.in_channels} "
                       "is outside the native path")

    def build(tape, xa):
        return tape.gn_conv(xa, "c", k, s, standardize=standardize)

    return subgraph.run(build, x, [("c.weight", m.weight)], std=standardize)


def conv3x3x3(in_planes, out_planes, kernel_size=(3, 3, 3), stride=(1, 1, 1), padding=1, dilation=1, bias=False,
              weight_std=False):
    """Reference unet3D.py:30-35."""
    if weight_std:
        return Conv3d(in_planes, out_planes, kernel_size=kernel_size, stride=stride, padding=padding,
                      dilation=dilation, bias=bias)
    return nn.Conv3d(in_planes, out_planes, kernel_size=kernel_size, stride=stride, padding=padding,
                     dilation=dilation, bias=bias)


class NoBottleneck(nn.Module):
    """Pre-activation residual block, reference unet3D.py:40-73 (same submodule names)."""

    def __init__(self, inplanes, planes, stride=1, dilation=1, downsample=None, fist_dilation=1, multi_grid=1,
                 weight_std=False, group=16):
        super().__init__()
        self.weight_std = weight_std
        self.gn1 = nn.GroupNorm(group, inplanes)
        self.conv1 = conv3x3x3(inplanes, planes, kernel_size=(3, 3, 3), stride=stride, padding=(1, 1, 1),
                               dilation=dilation * multi_grid, bias=False, weight_std=self.weight_std)
        self.relu = nn.ReLU(inplace=in_place)
        self.gn2 = nn.GroupNorm(group, planes)
        self.conv2 = conv3x3x3(planes, planes, kernel_size=(3, 3, 3), stride=1, padding=(1, 1, 1),
                               dilation=dilation * multi_grid, bias=False, weight_std=self.weight_std)
        self.downsample = downsample
        self.dilation = dilation
        self.stride = stride
        self.group = group

    def forward(self, x):
        s = self.stride if isinstance(self.stride, int) else self.stride[0]
        G = self.group

        def build(tape, xa):
            return tape.block(xa, "", s, G)

        return subgraph.run(build, x, list(self.named_parameters()), std=self.weight_std)


def _make_layer(model, block, inplanes, planes, blocks, stride=(1, 1, 1), dilation=1, multi_grid=1, group=16,
                ds_group=16):
    """Shared _make_layer (reference :1666-1686 / :1538-1564)."""
    downsample = None
    if stride[0] != 1 or stride[1] != 1 or stride[2] != 1 or inplanes != planes:
        downsample = nn.Sequential(
            nn.GroupNorm(ds_group, inplanes),
            nn.ReLU(inplace=in_place),
            conv3x3x3(inplanes, planes, kernel_size=(1, 1, 1), stride=stride, padding=0, weight_std=model.weight_std),
        )
    layers = []
    gm = lambda index, grids: grids[index % len(grids)] if isinstance(grids, tuple) else 1  # noqa: E731
    layers.append(block(inplanes, planes, stride, dilation=dilation, downsample=downsample,
                        multi_grid=gm(0, multi_grid), weight_std=model.weight_std, group=group))
    for i in range(1, blocks):
        layers.append(block(planes, planes, dilation=dilation, multi_grid=gm(i, multi_grid),
                            weight_std=model.weight_std, group=group))
    return nn.Sequential(*layers)


class _TrunkMixin:
    """Builds the conv1 / layer0-4 / fusionConv / decoder / precls_conv modules with reference names."""

    def _build_trunk(self, in_channel, f, layers, group, fusion_group, head_group, ncls, conv0=False):
        if conv0:
            self.conv0 = conv3x3x3(in_channel, f, stride=[2, 2, 2], weight_std=self.weight_std)
            self.conv1 = conv3x3x3(f, f, stride=[1, 1, 1], weight_std=self.weight_std)
        else:
            self.conv1 = conv3x3x3(in_channel, f, stride=[1, 1, 1], weight_std=self.weight_std)
        mk = lambda cin, cout, n, s: _make_layer(self, NoBottleneck, cin, cout, n, stride=s, group=group,  # noqa
                                                 ds_group=group)
        self.layer0 = mk(f, f, layers[0], (1, 1, 1))
        self.layer1 = mk(f, 2 * f, layers[1], (2, 2, 2))
        self.layer2 = mk(2 * f, 4 * f, layers[2], (2, 2, 2))
        self.layer3 = mk(4 * f, 8 * f, layers[3], (2, 2, 2))
        self.layer4 = mk(8 * f, 8 * f, layers[4], (2, 2, 2))
        self.fusionConv = nn.Sequential(
            nn.GroupNorm(fusion_group, 8 * f),
            nn.ReLU(inplace=in_place),
            conv3x3x3(8 * f, 8 * f, kernel_size=(1, 1, 1), padding=(0, 0, 0), weight_std=self.weight_std),
        )
        self.upsamplex2 = nn.Upsample(scale_factor=2, mode="trilinear")
        self.x8_resb = mk(8 * f, 4 * f, 1, (1, 1, 1))
        self.x4_resb = mk(4 * f, 2 * f, 1, (1, 1, 1))
        self.x2_resb = mk(2 * f, f, 1, (1, 1, 1))
        self.x1_resb = mk(f, f, 1, (1, 1, 1))
        self.precls_conv = nn.Sequential(
            nn.GroupNorm(head_group, f),
            nn.ReLU(inplace=in_place),
            nn.Conv3d(f, ncls, kernel_size=1),
        )
        self._u3d_cfg = trunk.TrunkCfg(layers=tuple(layers), groups=group, fusion_groups=fusion_group,
                                       head_groups=head_group, conv0=conv0, final_up=conv0,
                                       weight_std=bool(self.weight_std))

    def _make_layer(self, block, inplanes, planes, blocks, stride=(1, 1, 1), dilation=1, multi_grid=1):
        return _make_layer(self, block, inplanes, planes, blocks, stride, dilation, multi_grid,
                           group=self._u3d_cfg.groups if hasattr(self, "_u3d_cfg") else 16)

    def _trunk_params(self):
        return [(n, p) for n, p in self.named_parameters()
                if not n.startswith(("GAP.", "controller."))]

    def _run(self, x):
        return trunk.run_trunk(self._u3d_cfg, x, self._trunk_params(), getattr(self, "compute_dtype", None))


class unet3D_baseline(_TrunkMixin, nn.Module):
    """Reference unet3D.py:584-718. forward(input, mask=None) -> train: (logits, [], []); eval: logits."""

    def __init__(self, layers, num_classes=12, weight_std=False, ema=False, use_cm=[True, True, True],  # noqa: B006
                 deep_up=False):
        super().__init__()
        self.inplanes = 128
        self.weight_std = weight_std
        self.num_classes = num_classes
        self.use_cm = use_cm
        self.alpha = 0.01
        self.deep_up = deep_up
        self._build_trunk(1, 32, layers, 16, 16, 16, num_classes)
        self.upsamplex3 = nn.Upsample(scale_factor=4, mode="trilinear")
        self.upsamplex4 = nn.Upsample(scale_factor=8, mode="trilinear")
        if ema:
            for param in self.parameters():
                param.detach_()

    def forward(self, input, mask=None):
        logits = self._run(input)
        if self.training:
            return logits, [], []
        return logits


class unet3D_g(_TrunkMixin, nn.Module):
    """Reference unet3D.py:1507-1623 (the refiner / light variant): stride-2 conv0, GN(4) blocks,
    GN(init/2) fusion, GN(init/4) head, final x2 upsample of the logits."""

    def __init__(self, layers, num_classes=3, weight_std=False, in_channel=2, init_filter=32):
        super().__init__()
        self.inplanes = 128
        self.weight_std = weight_std
        self.init_filter = init_filter
        self._build_trunk(in_channel, init_filter, layers, 4, init_filter // 2, init_filter // 4, num_classes,
                          conv0=True)

    def forward(self, input, _=None):
        return self._run(input)


class unet3D(_TrunkMixin, nn.Module):
    """Reference unet3D.py:1625-1806: trunk + DynConv 8,8,2 head conditioned on the task id."""

    def __init__(self, layers, num_classes=3, weight_std=False, in_channel=1, init_filter=32):
        super().__init__()
        self.inplanes = 128
        self.weight_std = weight_std
        self.init_filter = init_filter
        self._build_trunk(in_channel, init_filter, layers, 16, 16, 16, 8)
        self.GAP = nn.Sequential(nn.GroupNorm(16, 256), nn.ReLU(inplace=in_place), torch.nn.AdaptiveAvgPool3d((1, 1, 1)))
        self.controller = nn.Conv3d(256 + 7, 162, kernel_size=1, stride=1, padding=0)

    def forward(self, input, task_id):
        from u3d import dynhead
        return dynhead.run_unet3d(self, input, task_id)


def UNet3D(num_classes=1, weight_std=False):
    """Reference factory unet3D.py:1808-1811."""
    print("Using DynConv 8,8,2")
    return unet3D([1, 2, 2, 2, 2], num_classes, weight_std)


def _next_row(name, row):
    def ctor(*a, **k):
        raise NotImplementedError(f"{name}: method-specific head, SURVEY.md §8(f) row {row} — not built in this round")
    ctor.__name__ = name
    return ctor


class EAM(nn.Module):
    """Reference unet3D.py:142-212 (same parameters: kv, q, proj, norm2, norm3). Inside unet3D_with_feam3 its
    attention map runs natively (u3d.feam: only ``attn`` is used there, :1134); called on its own it raises."""

    def __init__(self, dim, input_resolution, num_heads, mlp_ratio=4., qkv_bias=True, qk_scale=None, drop=0.,
                 attn_drop=0., drop_path=0., norm_layer=nn.LayerNorm, upsample=None, use_checkpoint=False):
        super().__init__()
        self.dim = dim
        self.input_resolution = input_resolution
        self.use_checkpoint = use_checkpoint
        self.num_heads = num_heads
        head_dim = dim // num_heads
        self.scale = qk_scale or head_dim ** -0.5
        self.kv = nn.Linear(dim, dim * 2, bias=False)
        self.q = nn.Linear(dim, dim, bias=False)
        self.softmax = nn.Softmax(dim=-1)
        self.proj = nn.Linear(dim, dim)
        self.norm2 = norm_layer(dim)
        self.norm3 = norm_layer(dim)

    def forward(self, x, modality_token):
        raise U3DError("EAM: the native path runs it inside unet3D_with_feam3 (u3d.feam); standalone use is not "
                       "on the hot path")


class unet3D_with_feam3(_TrunkMixin, nn.Module):
    """Reference unet3D.py:938-1190 (the model train_amos_atlas_final.py:118 trains): the trunk + deep-supervision
    heads deepout1-3 + EAM attention maps against EMA class tokens. forward(input, mask=None) -> train:
    (logits, atten_map[<=3], deep_map[3], feature_stored[3]); eval: logits. Batch 1 when use_cm (the reference's
    EAM reshapes with the token's batch of 1 and raises otherwise)."""

    def __init__(self, layers, num_classes=12, weight_std=False, ema=False, use_cm=[True, True, True],  # noqa: B006
                 deep_up=False):
        self.inplanes = 128
        self.weight_std = weight_std
        self.num_classes = num_classes
        self.use_cm = use_cm
        self.alpha = 0.01
        self.deep_up = deep_up
        super().__init__()
        mk = lambda cin, cout, n, s: _make_layer(self, NoBottleneck, cin, cout, n, stride=s)  # noqa: E731
        self.conv1 = conv3x3x3(1, 32, stride=[1, 1, 1], weight_std=self.weight_std)
        self.layer0 = mk(32, 32, layers[0], (1, 1, 1))
        self.layer1 = mk(32, 64, layers[1], (2, 2, 2))
        self.layer2 = mk(64, 128, layers[2], (2, 2, 2))
        self.layer3 = mk(128, 256, layers[3], (2, 2, 2))
        self.layer4 = mk(256, 256, layers[4], (2, 2, 2))
        self.fusionConv = nn.Sequential(
            nn.GroupNorm(16, 256), nn.ReLU(inplace=in_place),
            conv3x3x3(256, 256, kernel_size=(1, 1, 1), padding=(0, 0, 0), weight_std=self.weight_std))
        self.upsamplex2 = nn.Upsample(scale_factor=2, mode="trilinear")
        self.upsamplex3 = nn.Upsample(scale_factor=4, mode="trilinear")
        self.upsamplex4 = nn.Upsample(scale_factor=8, mode="trilinear")
        head = lambda c: nn.Sequential(nn.GroupNorm(16, c), nn.ReLU(inplace=in_place),  # noqa: E731
                                       nn.Conv3d(c, num_classes, kernel_size=1))
        self.x8_resb = mk(256, 128, 1, (1, 1, 1))
        self.deepout1 = head(128)
        self.eam84 = EAM(128, input_resolution=None, num_heads=4)
        self.x4_resb = mk(128, 64, 1, (1, 1, 1))
        self.deepout2 = head(64)
        self.eam42 = EAM(64, input_resolution=None, num_heads=4)
        self.x2_resb = mk(64, 32, 1, (1, 1, 1))
        self.deepout3 = head(32)
        self.eam21 = EAM(32, input_resolution=None, num_heads=4)
        self.x1_resb = mk(32, 32, 1, (1, 1, 1))
        self.precls_conv = head(32)
        # class tokens: plain tensors (not parameters / buffers, so not in the state_dict), :1016-1021
        self.class_token1 = torch.randn(num_classes - 1, 128)
        self.class_token2 = torch.randn(num_classes - 1, 64)
        self.class_token3 = torch.randn(num_classes - 1, 32)
        self._u3d_cfg = trunk.TrunkCfg(layers=tuple(layers), weight_std=bool(self.weight_std))
        if ema:
            for param in self.parameters():
                param.detach_()

    def renew_token(self, features, mask):
        """EMA update of the class tokens from the stored features (:1051-1068), on the device."""
        from u3d import feam
        dev = mask.device
        self.class_token1 = self.class_token1.to(dev)
        self.class_token2 = self.class_token2.to(dev)
        self.class_token3 = self.class_token3.to(dev)
        feam.renew_token([self.class_token1, self.class_token2, self.class_token3], features, mask,
                         self.num_classes, self.alpha)

    def forward(self, input, mask=None):
        from u3d import feam
        self.class_token1 = self.class_token1.to(input.device)
        self.class_token2 = self.class_token2.to(input.device)
        self.class_token3 = self.class_token3.to(input.device)
        return feam.run_feam3(self, input)


class unet3D_with_feam2(unet3D_with_feam3):
    """Reference unet3D.py:721-936 — the model evaluate_amos.py:571 builds. Same modules as unet3D_with_feam3; the
    class tokens are nn.Parameters (in the state_dict, registered last, :788-793) updated INSIDE forward in train
    mode (each level before its attention). forward(input, mask=None) -> train: (logits, atten_map, deep_map);
    eval: logits. As in the reference, a train-mode forward with a mask updates the tokens in place, which
    autograd refuses while they require grad (it works with ema=True), and mask=None fails at ``(mask == l+1)``."""

    def __init__(self, layers, num_classes=12, weight_std=False, ema=False, use_cm=[True, True, True],  # noqa: B006
                 deep_up=False):
        super().__init__(layers, num_classes, weight_std, False, use_cm, deep_up)
        self.class_token1 = nn.Parameter(torch.randn(num_classes - 1, 128))
        self.class_token2 = nn.Parameter(torch.randn(num_classes - 1, 64))
        self.class_token3 = nn.Parameter(torch.randn(num_classes - 1, 32))
        if ema:
            for param in self.parameters():
                param.detach_()

    def _trunk_named(self):
        return [(n, p) for n, p in self.named_parameters() if not n.startswith("class_token")]

    def forward(self, input, mask=None):
        from u3d import feam
        if not self.training:
            return feam.run_feam3(self, input)
        if mask is None:
            raise AttributeError("'bool' object has no attribute 'sum'")  # (None == l+1).sum(), unet3D.py:870
        outs = feam.run_feam3(self, input, renew=(mask, self.num_classes, self.alpha))
        return outs[0], outs[1], outs[2]


# Method-specific variants and discriminators: next rows, not on the trunk path.
unet3D_with_feam = _next_row("unet3D_with_feam", "f2")
unet3D_with_eam = _next_row("unet3D_with_eam", "f2")
unet3D_with_eam_baseline = _next_row("unet3D_with_eam_baseline", "f2")
unet3D_with_deepsup = _next_row("unet3D_with_deepsup", "f2")
get_style_discriminator = _next_row("get_style_discriminator", "out-of-scope")
get_style_discriminator_output = _next_row("get_style_discriminator_output", "out-of-scope")
deep_style_discriminator_output = _next_row("deep_style_discriminator_output", "out-of-scope")
norm_style_discriminator_output = _next_row("norm_style_discriminator_output", "out-of-scope")
