"""unet3D_with_feam3 on the native executor (reference unet3D.py:938-1190), forward and backward.

Forward (one autograd Function around the whole model): the shared trunk tape (conv1 .. x1_resb, precls_conv), plus
at each of the x8 / x4 / x2 decoder levels
  * deepout{1,2,3} = GN(16) -> ReLU -> Conv3d 1^3 + bias (:969-993, same fused GN-prologue conv as precls_conv);
  * the EAM attention map against the detached class token (:1131-1175): u3d_eam_prep (token side: LN3, q, M) and
    u3d_eam_attn_fwd (per-voxel LN2 + Nt x C GEMV, written NCDHW), x8/x4/x2 trilinear-upsampled to full size when
    deep_up (u3d_upsample_trilinear);
  * a detached copy of the feature (feature_stored, :1129).
Backward: every output gradient that autograd hands in (unused outputs arrive as None and cost nothing) is pushed
through the same kernels' backward (u3d_upsample_trilinear_bwd, u3d_eam_attn_bwd, u3d_eam_param_bwd, the 1^3 head
backward), accumulated into the decoder features' gradients, then the trunk tape replays.
renew_token (:1051-1068) is u3d_renew_token on the stored features, in place on the device class tokens.
"""
import torch

from . import ops, trunk
from ._lib import call, query
from .ddp import current_sink

EAM_KEYS = ("eam84", "eam42", "eam21")
UP_SCALE = (8, 4, 2)   # upsamplex4 / upsamplex3 / upsamplex2 for deep_up (:1138, :1156, :1175)
NUM_HEADS = 4          # EAM(dim, num_heads=4) (:975, :985, :996)


def _eam_shape_error(n, v, c):
    """The reference's kv reshape uses the token's batch of 1 (unet3D.py:189, :198): B > 1 fails there."""
    return RuntimeError(f"shape '[1, {v}, 2, {NUM_HEADS}, {c // NUM_HEADS}]' is invalid for input of size "
                        f"{n * v * 2 * c}")


def upsample_trilinear(x, s):
    """NCDHW fp32 [n, c, d, h, w] -> [n, c, sd, sh, sw] (nn.Upsample(scale_factor=s, mode='trilinear'))."""
    n, c, d, h, w = x.shape
    y = torch.empty((n, c, d * s, h * s, w * s), dtype=torch.float32, device=x.device)
    call("u3d_upsample_trilinear", x.data_ptr(), n * c, d, h, w, s, y.data_ptr(), ops._stream())
    return y


def upsample_trilinear_bwd(dy, in_shape, s):
    n, c, d, h, w = in_shape
    if dy.dtype != torch.float32 or not dy.is_contiguous():
        dy = dy.float().contiguous()
    dx = torch.empty(in_shape, dtype=torch.float32, device=dy.device)
    ws = torch.empty(query("u3d_upsample_trilinear_bwd_ws_floats", n * c, d, h, w, s), dtype=torch.float32,
                     device=dy.device)
    call("u3d_upsample_trilinear_bwd", dy.data_ptr(), n * c, d, h, w, s, dx.data_ptr(), 0, ws.data_ptr(),
         ops._stream())
    return dx


def eam_op(tape, f, key, token, up):
    """EAM attention map of decoder feature ``f`` (Act, NDHWC) against ``token`` [nt, C] -> Act holding the NCDHW
    fp32 map [n, nt, d, h, w] (upsampled x``up`` when up > 1). Records its backward on the tape."""
    P = tape.P
    x = f.t
    n, d, h, w, c = x.shape
    v = d * h * w
    if n != 1:
        raise _eam_shape_error(n, v, c)
    nt = token.shape[0]
    dev = x.device
    tok = token.detach().float().contiguous()
    wk = P[key + ".kv.weight"]            # [2c, c]: rows 0..c-1 = k (kv reshape (2, heads, c/heads), :198-199)
    wq = P[key + ".q.weight"]
    g2, b2 = P[key + ".norm2.weight"], P[key + ".norm2.bias"]
    g3, b3 = P[key + ".norm3.weight"], P[key + ".norm3.bias"]
    zhat, q, M = (torch.empty((nt, c), dtype=torch.float32, device=dev) for _ in range(3))
    inv_h = 1.0 / NUM_HEADS
    st = ops._stream()
    call("u3d_eam_prep", tok.data_ptr(), nt, c, g3.data_ptr(), b3.data_ptr(), wq.data_ptr(), wk.data_ptr(), inv_h,
         zhat.data_ptr(), q.data_ptr(), M.data_ptr(), st)
    att = torch.empty((n, nt, d, h, w), dtype=torch.float32, device=dev)
    call("u3d_eam_attn_fwd", ops.dt_code(x.dtype), x.data_ptr(), n, v, c, g2.data_ptr(), b2.data_ptr(), M.data_ptr(),
         nt, att.data_ptr(), st)
    out = trunk.Act(upsample_trilinear(att, up) if up > 1 else att)
    if tape.record:
        def bwd():
            g = out.grad
            if g is None:
                return
            g = upsample_trilinear_bwd(g, tuple(att.shape), up) if up > 1 else g.float().contiguous()
            part = torch.empty(query("u3d_eam_attn_bwd_part_floats", n, v, c, nt), dtype=torch.float32, device=dev)
            dM = torch.empty((nt, c), dtype=torch.float32, device=dev)
            dg2 = tape.grad_out(key + ".norm2.weight", g2)
            db2 = tape.grad_out(key + ".norm2.bias", b2)
            acc = f.grad is not None
            dx = f.grad if acc else torch.empty_like(x)
            s = ops._stream()
            call("u3d_eam_attn_bwd", ops.dt_code(x.dtype), x.data_ptr(), n, v, c, g2.data_ptr(), b2.data_ptr(),
                 M.data_ptr(), nt, g.data_ptr(), dx.data_ptr(), int(acc), part.data_ptr(), dM.data_ptr(),
                 dg2.data_ptr(), db2.data_ptr(), 0, s)
            f.grad = dx
            dwq = tape.grad_out(key + ".q.weight", wq)
            dkv = tape.grad_out(key + ".kv.weight", wk)
            dg3 = tape.grad_out(key + ".norm3.weight", g3)
            db3 = tape.grad_out(key + ".norm3.bias", b3)
            dq_ws, dz_ws = torch.empty((nt, c), dtype=torch.float32, device=dev), torch.empty_like(dM)
            call("u3d_eam_param_bwd", dM.data_ptr(), nt, c, zhat.data_ptr(), g3.data_ptr(), b3.data_ptr(),
                 wq.data_ptr(), wk.data_ptr(), q.data_ptr(), inv_h, dq_ws.data_ptr(), dz_ws.data_ptr(),
                 dwq.data_ptr(), dkv.data_ptr(), dg3.data_ptr(), db3.data_ptr(), 0, s)
            for nm in (".norm2.weight", ".norm2.bias", ".q.weight", ".kv.weight", ".norm3.weight", ".norm3.bias"):
                tape.grad_done(key + nm)
        tape.ops.append(bwd)
    return out


def _feam3_forward(tape, cfg, x, tokens, use_cm, deep_up, heads=True, renew=None):
    """renew = (mask, num_classes, alpha): unet3D_with_feam2's in-forward class-token update of each level, before
    that level's attention (unet3D.py:869-878, 896-903, 919-926)."""
    f, _ = tape.trunk(x, cfg)
    lg = tape.head(f, cfg)
    att, deep, feats = [], [], []
    if heads:
        for k in range(3):
            fk = tape.dec[k]
            deep.append(tape.gn_conv(fk, f"deepout{k + 1}.2", 1, 1, gn_key=f"deepout{k + 1}.0", G=16, bias=True,
                                     out_f32=True, standardize=False))
            feats.append(fk.t.detach().clone())
            if renew is not None:
                renew_token([tokens[k]], [fk.t.permute(0, 4, 1, 2, 3)], renew[0], renew[1], renew[2])
            if use_cm[k]:
                att.append(eam_op(tape, fk, EAM_KEYS[k], tokens[k], UP_SCALE[k] if deep_up else 1))
    return lg, att, deep, feats


def _ncdhw(t):
    return t.permute(0, 4, 1, 2, 3)


class _Feam3Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, cfg, dtype, use_cm, deep_up, names, x, tokens, *tensors):
        ctx.set_materialize_grads(False)
        P = dict(zip(names, tensors))
        tape = trunk.Tape(P, dtype, record=True)
        tape.sink = current_sink()
        if tape.sink is not None:
            tape.sink.begin()
        lg, att, deep, feats = _feam3_forward(tape, cfg, x, tokens, use_cm, deep_up)
        ctx.state = (tape, lg, att, deep)
        ctx.names = names
        ctx.n_att = len(att)
        fo = [_ncdhw(ft) for ft in feats]
        ctx.mark_non_differentiable(*fo)
        return tuple([_ncdhw(lg.t)] + [a.t for a in att] + [_ncdhw(d.t) for d in deep] + fo)

    @staticmethod
    def backward(ctx, *grads):
        tape, lg, att, deep = ctx.state
        na = ctx.n_att
        g_lg = grads[0]
        for a, g in zip(att, grads[1:1 + na]):
            a.grad = g.contiguous() if g is not None else None
        for d, g in zip(deep, grads[1 + na:4 + na]):
            d.grad = g.permute(0, 2, 3, 4, 1).float().contiguous() if g is not None else None
        if g_lg is None:
            g_lg = torch.zeros(lg.t.shape, dtype=torch.float32, device=lg.t.device)
        else:
            g_lg = g_lg.permute(0, 2, 3, 4, 1).float().contiguous()
        tape.backward(lg, g_lg)
        if tape.sink is not None:
            tape.sink.finish()
        pg = [tape.pgrad.get(nm) for nm in ctx.names]
        if tape.sink is not None:
            pg = tape.sink.returned(ctx.names, pg)
        ctx.state = None
        return (None, None, None, None, None, None, None, *pg)


def run_feam3(model, x, renew=None):
    """model: unet3D.unet3D_with_feam3 (or _feam2). Returns train: (logits, atten_map, deep_map, feature_stored);
    eval: logits."""
    ops.require_device(x)
    cfg = model._u3d_cfg
    dtype = trunk.compute_dtype(getattr(model, "compute_dtype", None))
    x = x.float().contiguous()
    tokens = [model.class_token1, model.class_token2, model.class_token3]
    use_cm = tuple(bool(u) for u in model.use_cm)
    named = list(model.named_parameters())
    if not model.training:
        with torch.no_grad():
            tape = trunk.Tape(dict(named), dtype, record=False)
            lg, _, _, _ = _feam3_forward(tape, cfg, x, tokens, use_cm, model.deep_up, heads=False)
        return _ncdhw(lg.t)
    if torch.is_grad_enabled() and any(p.requires_grad for _, p in named):
        if renew is not None:
            raise RuntimeError("a leaf Variable that requires grad is being used in an in-place operation.")
        outs = _Feam3Fn.apply(cfg, dtype, use_cm, bool(model.deep_up), [nm for nm, _ in named], x, tokens,
                              *[p for _, p in named])
    else:
        with torch.no_grad():
            tape = trunk.Tape(dict(named), dtype, record=False)
            lg, att, deep, feats = _feam3_forward(tape, cfg, x, tokens, use_cm, model.deep_up, renew=renew)
        outs = [_ncdhw(lg.t)] + [a.t for a in att] + [_ncdhw(d.t) for d in deep] + [_ncdhw(ft) for ft in feats]
    na = sum(use_cm)
    return outs[0], list(outs[1:1 + na]), list(outs[1 + na:4 + na]), list(outs[4 + na:7 + na])


def renew_token(tokens, features, mask, num_classes, alpha):
    """u3d_renew_token per level (unet3D.py:1051-1068). tokens: device fp32 [nc-1, C] tensors, updated in place."""
    mask = mask.float().contiguous()
    ops.require_device(mask, *tokens)
    n, _, md, mh, mw = mask.shape
    for tok, feat in zip(tokens, features):
        nb, c, d, h, w = feat.shape
        if nb != n:
            raise RuntimeError(f"renew_token: feature batch {nb} != mask batch {n}")
        v = d * h * w
        st = feat.stride()
        if st[1] == 1 and st[4] == c and st[0] == v * c:       # NCDHW view of NDHWC storage (our features)
            sv, sc = c, 1
        elif feat.is_contiguous():                           # plain NCDHW
            sv, sc = 1, v
        else:
            feat = feat.contiguous()
            sv, sc = 1, v
        if feat.dtype not in (torch.float32, torch.bfloat16):
            feat = feat.float()
        ops.require_device(feat)
        ws = ops.WS.get(query("u3d_renew_token_ws_bytes", n, d, h, w, num_classes, c), feat.device, slot=6)
        call("u3d_renew_token", ops.dt_code(feat.dtype), feat.data_ptr(), sv, sc, n, d, h, w, c, mask.data_ptr(),
             md, mh, mw, num_classes, tok.shape[0], float(alpha), tok.data_ptr(), ws.data_ptr(), ops._stream())
