"""MixFormer RGB-T forward, CPU restatement in plain PyTorch fp32 (oracle; test infrastructure only).

Functional restatement, driven by a state_dict with the reference's key names, of:
  two-stream   MixFormer_RGBT.forward           lib/models/mixformer_vit_rgbt/mixformer.py:366-395
  shared       MixFormer_RGBT.forward           mixformer_shared.py:400-424 (modalities batch-stacked)
  asym         MixFormer_RGBT.forward           asymmetric_shared.py:349-368 (cross-modal MAM)
  asym_online  MixFormer_RGBT_OnlineScore.fwd   asymmetric_shared_online.py:351-413 (+ SPM)
  rgb          MixFormer.forward (RGB only)     lib/models/mixformer_vit/mixformer.py:294-305, :323-337
               (one VisionTransformer, :234-270, then the corner head on its search tokens)
with the pieces they share:
  PatchEmbed / pos-embed / token concat          mixformer.py:29-34, :237-248
  MAM attention (template->template, search->all) mixformer.py:52-78; asymmetric_shared.py:55-104
  pre-LN Block (eps 1e-6), timm Mlp (GELU erf)   mixformer.py:136-139; mixformer_shared.py:143-159
  Attention_Fusion_Bimodal_LNSpecific            fusion_utils.py:243-279
  DeformableAttentionFusion_LNSpecific + layer    deformable_encoder_lnspecific.py:70-160, :170-186
  MSDeformAttn_Bimodal                           ops/modules/ms_deform_attn_bimodal.py:83-130
  PositionEmbeddingSine(256, normalize)          position_encoding.py:34-54
  Pyramid_Corner_Predictor (BN eval) + soft-argmax mixformer_cvt/head.py:147-212
  box_xyxy_to_cxcywh / cxcywh_to_xyxy            lib/utils/box_ops.py
  ScoreDecoder (scale 768^-1/2)                  mixformer_cvt/score_decoder.py:32-66
The op order follows the reference so that fp32 results agree to ~1e-6.
"""
import math

import numpy as np
import torch
import torch.nn.functional as F

from .msda import ms_deform_attn
from .prroi import prroi_pool2d

VARIANTS = ("rgbt", "shared", "asym", "asym_online", "asym_ce", "rgb")
CE_LOC, CE_KEEP = (3, 6, 9), (0.7, 0.7, 0.7)  # lib/config/asymmetric_shared_ce/config.py:23-24


# ----------------------------------------------------------------------------- helpers
def _lin(sd, name, x):
    return F.linear(x, sd[name + ".weight"], sd[name + ".bias"])


def _ln(sd, name, x, eps):
    return F.layer_norm(x, (x.shape[-1],), sd[name + ".weight"], sd[name + ".bias"], eps)


def _mlp(sd, pre, x):
    return _lin(sd, pre + ".fc2", F.gelu(_lin(sd, pre + ".fc1", x)))


def _patch_embed(sd, pre, img):
    x = F.conv2d(img, sd[pre + "patch_embed.proj.weight"], sd[pre + "patch_embed.proj.bias"], stride=16)
    return x.flatten(2).transpose(1, 2).contiguous()


def _tokens(sd, pre, t, o, s):
    xt = _patch_embed(sd, pre, t) + sd[pre + "pos_embed_t"]
    xo = _patch_embed(sd, pre, o) + sd[pre + "pos_embed_t"]
    xs = _patch_embed(sd, pre, s) + sd[pre + "pos_embed_s"]
    return torch.cat([xt, xo, xs], dim=1)


def _heads(x, B, N, H):
    C = x.shape[-1] // 3
    return x.reshape(B, N, 3, H, C // H).permute(2, 0, 3, 1, 4)


def _sdpa(q, k, v, scale):
    a = (q @ k.transpose(-2, -1)) * scale
    return a.softmax(dim=-1) @ v


def mam_attention(qkv_w, qkv_b, proj_w, proj_b, x, n_t, num_heads):
    """Standard MAM (mixformer.py:52-78): template queries see the n_t template keys,
    search queries see all keys."""
    B, N, C = x.shape
    q, k, v = _heads(F.linear(x, qkv_w, qkv_b), B, N, num_heads).unbind(0)
    scale = (C // num_heads) ** -0.5
    x_mt = _sdpa(q[:, :, :n_t], k[:, :, :n_t], v[:, :, :n_t], scale)
    x_s = _sdpa(q[:, :, n_t:], k, v, scale)
    out = torch.cat([x_mt, x_s], dim=2).transpose(1, 2).reshape(B, N, C)
    return F.linear(out, proj_w, proj_b)


def mam_attention_asym(qkv_w, qkv_b, proj_w, proj_b, x_v, x_i, n_t, num_heads):
    """Cross-modal asymmetric MAM (asymmetric_shared.py:55-104): search_m attends
    [template_V | template_I | search_m]."""
    B, N, C = x_v.shape
    qkv = F.linear(torch.cat([x_v, x_i], 0), qkv_w, qkv_b).reshape(2 * B, N, 3, num_heads, C // num_heads)
    qV, kV, vV = qkv[:B].permute(2, 0, 3, 1, 4).unbind(0)
    qI, kI, vI = qkv[B:].permute(2, 0, 3, 1, 4).unbind(0)
    scale = (C // num_heads) ** -0.5
    k_mt = torch.cat([kV[:, :, :n_t], kI[:, :, :n_t]], 2)
    v_mt = torch.cat([vV[:, :, :n_t], vI[:, :, :n_t]], 2)
    x_mt_V = _sdpa(qV[:, :, :n_t], kV[:, :, :n_t], vV[:, :, :n_t], scale)
    x_mt_I = _sdpa(qI[:, :, :n_t], kI[:, :, :n_t], vI[:, :, :n_t], scale)
    x_s_V = _sdpa(qV[:, :, n_t:], torch.cat([k_mt, kV[:, :, n_t:]], 2), torch.cat([v_mt, vV[:, :, n_t:]], 2), scale)
    x_s_I = _sdpa(qI[:, :, n_t:], torch.cat([k_mt, kI[:, :, n_t:]], 2), torch.cat([v_mt, vI[:, :, n_t:]], 2), scale)
    xV = torch.cat([x_mt_V, x_s_V], 2).transpose(1, 2).reshape(B, N, C)
    xI = torch.cat([x_mt_I, x_s_I], 2).transpose(1, 2).reshape(B, N, C)
    out = F.linear(torch.cat([xV, xI], 0), proj_w, proj_b)
    return out[:B], out[B:]


# ----------------------------------------------------------------------------- backbones
def _vit_dims(sd, pre):
    C = sd[pre + "pos_embed_s"].shape[-1]
    depth = 0
    while (pre + "blocks.%d.mlp.fc1.weight" % depth) in sd:
        depth += 1
    return C, C // 64, depth, int(round(sd[pre + "pos_embed_t"].shape[1] ** 0.5)), int(round(sd[pre + "pos_embed_s"].shape[1] ** 0.5))


def _split_out(x, B, C, gt, gs):
    nt = gt * gt
    xt, xo, xs = torch.split(x, [nt, nt, gs * gs], dim=1)
    return (xt.transpose(1, 2).reshape(B, C, gt, gt), xo.transpose(1, 2).reshape(B, C, gt, gt),
            xs.transpose(1, 2).reshape(B, C, gs, gs))


def backbone_two_stream(sd, pre, t, o, s):
    """VisionTransformer.forward, mixformer.py:231-259 (one modality)."""
    C, H, depth, gt, gs = _vit_dims(sd, pre)
    x = _tokens(sd, pre, t, o, s)
    n_t = 2 * gt * gt
    for i in range(depth):
        b = pre + "blocks.%d." % i
        x = x + mam_attention(sd[b + "attn.qkv.weight"], sd[b + "attn.qkv.bias"], sd[b + "attn.proj.weight"],
                              sd[b + "attn.proj.bias"], _ln(sd, b + "norm1", x, 1e-6), n_t, H)
        x = x + _mlp(sd, b + "mlp", _ln(sd, b + "norm2", x, 1e-6))
    return _split_out(x, x.shape[0], C, gt, gs)


def backbone_shared(sd, pre, t, o, s):
    """mixformer_shared.py:143-159, :253-282; inputs are [v; i] stacked on the batch."""
    C, H, depth, gt, gs = _vit_dims(sd, pre)
    x = _tokens(sd, pre, t, o, s)
    B2 = x.shape[0]
    Bh = B2 // 2
    n_t = 2 * gt * gt
    for i in range(depth):
        b = pre + "blocks.%d." % i
        xn = torch.cat([_ln(sd, b + "norm1_v", x[:Bh], 1e-6), _ln(sd, b + "norm1_i", x[Bh:], 1e-6)], 0)
        x = x + mam_attention(sd[b + "attn.qkv.weight"], sd[b + "attn.qkv.bias"], sd[b + "attn.proj.weight"],
                              sd[b + "attn.proj.bias"], xn, n_t, H)
        xn = torch.cat([_ln(sd, b + "norm2_v", x[:Bh], 1e-6), _ln(sd, b + "norm2_i", x[Bh:], 1e-6)], 0)
        x = x + _mlp(sd, b + "mlp", xn)
    return _split_out(x, B2, C, gt, gs)


def backbone_asym(sd, pre, t, o, s):
    """asymmetric_shared.py:137-154, :236-266."""
    C, H, depth, gt, gs = _vit_dims(sd, pre)
    x = _tokens(sd, pre, t, o, s)
    B2 = x.shape[0]
    Bh = B2 // 2
    n_t = 2 * gt * gt
    x_v, x_i = x[:Bh], x[Bh:]
    for i in range(depth):
        b = pre + "blocks.%d." % i
        res = torch.cat([x_v, x_i], 0)
        a_v, a_i = mam_attention_asym(sd[b + "attn.qkv.weight"], sd[b + "attn.qkv.bias"], sd[b + "attn.proj.weight"],
                                      sd[b + "attn.proj.bias"], _ln(sd, b + "norm1_v", x_v, 1e-6),
                                      _ln(sd, b + "norm1_i", x_i, 1e-6), n_t, H)
        res = res + torch.cat([a_v, a_i], 0)
        x_v, x_i = res[:Bh], res[Bh:]
        xn = torch.cat([_ln(sd, b + "norm2_v", x_v, 1e-6), _ln(sd, b + "norm2_i", x_i, 1e-6)], 0)
        res = res + _mlp(sd, b + "mlp", xn)
        x_v, x_i = res[:Bh], res[Bh:]
    return _split_out(torch.cat([x_v, x_i], 0), B2, C, gt, gs)


def ce_attn_mean(q_v, q_i, k_v, k_i, n_t, scale, mask=None):
    """attn_t2s of Asym_Attention.forward(return_attention=True) (asymmetric_shared_ce.py:198-202),
    averaged over template queries and heads (candidate_elimination :81-92): softmax over
    [k_s_V | k_s_I] of [q_mt_V; q_mt_I], -> (B, 2 * lens_s) [RGB | TIR].  mask (B, 2 n_t) bool
    (ce_template_mask, e.g. ce_utils.py:14-38 CTR_POINT): only the masked queries' rows are averaged,
    attn[mask].view(bs, hn, -1, L) as :81-86."""
    q = torch.cat([q_v[:, :, :n_t], q_i[:, :, :n_t]], 2)
    k = torch.cat([k_v[:, :, n_t:], k_i[:, :, n_t:]], 2)
    a = ((q @ k.transpose(-2, -1)) * scale).softmax(dim=-1)
    if mask is not None:
        bs, hn, _, L = a.shape
        m = mask.to(torch.bool).unsqueeze(1).unsqueeze(-1).expand(-1, hn, -1, L)
        a = a[m].view(bs, hn, -1, L)
    return a.mean(dim=2).mean(dim=1)


def ce_select(attn_mean, x, n_t, keep_ratio, gidx, forced=None):
    """get_token_from_attn (asymmetric_shared_ce.py:22-46) for one modality: sort the search tokens'
    mean attention descending, keep the first ceil(keep_ratio * lens_s) (in that order) after the
    template tokens; gidx tracks their original search positions.  forced (B, keep): original
    positions to keep instead (test hook: replays another implementation's discrete choices)."""
    lens_s = x.shape[1] - n_t
    keep = math.ceil(keep_ratio * lens_s)
    if keep == lens_s:
        return x, gidx
    if forced is None:
        order = torch.sort(attn_mean, dim=1, descending=True)[1][:, :keep]
    else:
        inv = torch.full((gidx.shape[0], int(gidx.max()) + 1), -1, dtype=torch.long)
        inv.scatter_(1, gidx.long(), torch.arange(lens_s).repeat(gidx.shape[0], 1))
        order = inv.gather(1, torch.as_tensor(forced, dtype=torch.long)[:, :keep])
        assert bool((order >= 0).all()), "forced selection keeps a token pruned earlier"
    xs = x[:, n_t:].gather(1, order.unsqueeze(-1).expand(-1, -1, x.shape[2]))
    return torch.cat([x[:, :n_t], xs], 1), gidx.gather(1, order)


def backbone_asym_ce(sd, pre, t, o, s, stages=None, forced=None, mask=None):
    """asymmetric_shared_ce.py:228-282 (CE_Block_Shared), :372-424 (VisionTransformer.forward with
    _recover_search).  The elimination runs after a CE block's attention residual, before its MLP;
    pruned search positions come back as zero tokens.  `stages` (a list) receives the kept indices;
    mask = ce_template_mask (see ce_attn_mean)."""
    C, H, depth, gt, gs = _vit_dims(sd, pre)
    x = _tokens(sd, pre, t, o, s)
    B2 = x.shape[0]
    Bh = B2 // 2
    n_t = 2 * gt * gt
    N = gs * gs
    gidx = [torch.arange(N).repeat(Bh, 1), torch.arange(N).repeat(Bh, 1)]
    x_v, x_i = x[:Bh], x[Bh:]
    scale = (C // H) ** -0.5
    for i in range(depth):
        b = pre + "blocks.%d." % i
        n = x_v.shape[1]
        res = torch.cat([x_v, x_i], 0)
        xn_v, xn_i = _ln(sd, b + "norm1_v", x_v, 1e-6), _ln(sd, b + "norm1_i", x_i, 1e-6)
        a_v, a_i = mam_attention_asym(sd[b + "attn.qkv.weight"], sd[b + "attn.qkv.bias"], sd[b + "attn.proj.weight"],
                                      sd[b + "attn.proj.bias"], xn_v, xn_i, n_t, H)
        res = res + torch.cat([a_v, a_i], 0)
        x_v, x_i = res[:Bh], res[Bh:]
        if i in CE_LOC:
            qkv = F.linear(torch.cat([xn_v, xn_i], 0), sd[b + "attn.qkv.weight"], sd[b + "attn.qkv.bias"])
            q, k, _ = _heads(qkv, B2, n, H).unbind(0)
            am = ce_attn_mean(q[:Bh], q[Bh:], k[:Bh], k[Bh:], n_t, scale, mask)
            ls = n - n_t
            st = CE_LOC.index(i)
            fv, fi = forced[st] if forced is not None else (None, None)
            x_v, gidx[0] = ce_select(am[:, :ls], x_v, n_t, CE_KEEP[st], gidx[0], fv)
            x_i, gidx[1] = ce_select(am[:, ls:], x_i, n_t, CE_KEEP[st], gidx[1], fi)
            if stages is not None:
                stages.append((am, gidx[0].clone(), gidx[1].clone()))
        res = torch.cat([x_v, x_i], 0)
        xn = torch.cat([_ln(sd, b + "norm2_v", x_v, 1e-6), _ln(sd, b + "norm2_i", x_i, 1e-6)], 0)
        res = res + _mlp(sd, b + "mlp", xn)
        x_v, x_i = res[:Bh], res[Bh:]
    outs = []
    for xm, gm in ((x_v, gidx[0]), (x_i, gidx[1])):  # _recover_search: scatter back, zeros where pruned
        full = torch.zeros(Bh, N, C, dtype=xm.dtype)
        full.scatter_(1, gm.unsqueeze(-1).expand(-1, -1, C), xm[:, n_t:])
        outs.append(torch.cat([xm[:, :n_t], full], 1))
    return _split_out(torch.cat(outs, 0), B2, C, gt, gs)


# ----------------------------------------------------------------------------- fusion
def sine_pos_embed(B, C, H, W):
    """PositionEmbeddingSine(C/2, normalize=True), position_encoding.py:34-54, all-False mask."""
    npf = C // 2
    not_mask = torch.ones(B, H, W)
    y_embed = not_mask.cumsum(1, dtype=torch.float32)
    x_embed = not_mask.cumsum(2, dtype=torch.float32)
    eps = 1e-6
    scale = 2 * math.pi
    y_embed = (y_embed - 0.5) / (y_embed[:, -1:, :] + eps) * scale
    x_embed = (x_embed - 0.5) / (x_embed[:, :, -1:] + eps) * scale
    dim_t = torch.arange(npf, dtype=torch.float32)
    dim_t = 10000 ** (2 * (dim_t // 2) / npf)
    pos_x = x_embed[:, :, :, None] / dim_t
    pos_y = y_embed[:, :, :, None] / dim_t
    pos_x = torch.stack((pos_x[:, :, :, 0::2].sin(), pos_x[:, :, :, 1::2].cos()), dim=4).flatten(3)
    pos_y = torch.stack((pos_y[:, :, :, 0::2].sin(), pos_y[:, :, :, 1::2].cos()), dim=4).flatten(3)
    return torch.cat((pos_y, pos_x), dim=3).permute(0, 3, 1, 2)


def reference_points(H, W, B, L):
    """get_reference_points (deformable_encoder_lnspecific.py:170-186) with valid ratios 1."""
    refs = []
    for _ in range(L):
        ry, rx = torch.meshgrid(torch.linspace(0.5, H - 0.5, H), torch.linspace(0.5, W - 0.5, W), indexing="ij")
        ry = ry.reshape(-1)[None] / H
        rx = rx.reshape(-1)[None] / W
        refs.append(torch.stack((rx, ry), -1).expand(B, -1, -1))
    ref = torch.cat(refs, 1)
    return ref[:, :, None].expand(B, ref.shape[1], L, 2).contiguous()


def _gn(sd, name, x, groups=32):
    return F.group_norm(x, groups, sd[name + ".weight"], sd[name + ".bias"], 1e-5)


def _conv1x1(sd, name, x):
    return F.conv2d(x, sd[name + ".weight"], sd[name + ".bias"])


def msdeform_bimodal(sd, pre, query, ref, value_in, shapes, n_heads=8, n_levels=2, n_points=4):
    """MSDeformAttn_Bimodal.forward, ms_deform_attn_bimodal.py:83-130."""
    N, Lq, C = query.shape
    Lh = Lq // 2
    q_bi = torch.cat(torch.chunk(query, 2, 1), dim=2)
    value = _lin(sd, pre + "value_proj", value_in).view(N, value_in.shape[1], n_heads, C // n_heads)
    off = _lin(sd, pre + "sampling_offsets", q_bi).view(N, Lh, n_heads, n_levels, n_points, 2)
    off = torch.cat([off, off], 1)
    aw = _lin(sd, pre + "attention_weights", q_bi).view(N, Lh, n_heads, n_levels * n_points)
    aw = torch.cat([aw, aw], 1)
    aw = F.softmax(aw, -1).view(N, Lq, n_heads, n_levels, n_points)
    sh = torch.as_tensor(shapes, dtype=torch.long)
    normalizer = torch.stack([sh[..., 1], sh[..., 0]], -1)
    loc = ref[:, :, None, :, None, :] + off / normalizer[None, None, None, :, None, :]
    starts = [0]
    for h, w in shapes[:-1]:
        starts.append(starts[-1] + h * w)
    out = ms_deform_attn(value, shapes, starts, loc, aw)
    return _lin(sd, pre + "output_proj", out)


def fusion_lnspecific(sd, pre, in_v, in_i):
    """Attention_Fusion_Bimodal_LNSpecific.forward, fusion_utils.py:270-279."""
    b, c, h, w = in_v.shape
    av = _gn(sd, pre + "adjust_v.1", _conv1x1(sd, pre + "adjust_v.0", in_v))
    ai = _gn(sd, pre + "adjust_i.1", _conv1x1(sd, pre + "adjust_i.0", in_i))
    d = av.shape[1]
    fa = pre + "fusion_attention."
    pos = sine_pos_embed(b, d, h, w).flatten(2).transpose(1, 2)
    lvl = sd[fa + "level_embed"]
    src = torch.cat([av.flatten(2).transpose(1, 2), ai.flatten(2).transpose(1, 2)], 1)
    lpos = torch.cat([pos + lvl[0].view(1, 1, -1), pos + lvl[1].view(1, 1, -1)], 1)
    shapes = [(h, w), (h, w)]
    ref = reference_points(h, w, b, 2)
    n_layers = 0
    while (fa + "encoder.layers.%d.linear1.weight" % n_layers) in sd:
        n_layers += 1
    for li in range(n_layers):
        lp = fa + "encoder.layers.%d." % li
        src2 = msdeform_bimodal(sd, lp + "self_attn.", src + lpos, ref, src, shapes)
        src = src + src2
        s_v, s_i = torch.chunk(src, 2, 1)
        src = torch.cat([_ln(sd, lp + "norm1_v", s_v, 1e-5), _ln(sd, lp + "norm1_i", s_i, 1e-5)], 1)
        src2 = _lin(sd, lp + "linear2", F.relu(_lin(sd, lp + "linear1", src)))
        src = src + src2
        s_v, s_i = torch.chunk(src, 2, 1)
        src = torch.cat([_ln(sd, lp + "norm2_v", s_v, 1e-5), _ln(sd, lp + "norm2_i", s_i, 1e-5)], 1)
    o_v, o_i = torch.chunk(src, 2, 1)
    o_v = o_v.permute(0, 2, 1).reshape(b, -1, h, w)
    o_i = o_i.permute(0, 2, 1).reshape(b, -1, h, w)
    return _gn(sd, pre + "adjust_cat.1", _conv1x1(sd, pre + "adjust_cat.0", torch.cat([o_v, o_i], 1)))


# ----------------------------------------------------------------------------- head
def _cbr(sd, name, x):
    """conv() block: Conv3x3(bias) -> BatchNorm2d (eval) -> ReLU, head.py:7-20."""
    y = F.conv2d(x, sd[name + ".0.weight"], sd[name + ".0.bias"], padding=1)
    y = F.batch_norm(y, sd[name + ".1.running_mean"], sd[name + ".1.running_var"], sd[name + ".1.weight"],
                     sd[name + ".1.bias"], False, 0.0, 1e-5)
    return F.relu(y)


def _up(x, f):
    return F.interpolate(x, scale_factor=f)


def corner_score_maps(sd, pre, x):
    """Pyramid_Corner_Predictor.get_score_map, head.py:159-198."""
    maps = []
    for br in ("tl", "br"):
        x1 = _cbr(sd, pre + "conv1_" + br, x)
        x2 = _cbr(sd, pre + "conv2_" + br, x1)
        xu1 = _up(_cbr(sd, pre + "adjust1_" + br, x), 2) + _up(x2, 2)
        x3 = _cbr(sd, pre + "conv3_" + br, xu1)
        xu2 = _up(_cbr(sd, pre + "adjust2_" + br, x), 4) + _up(x3, 2)
        x4 = _cbr(sd, pre + "conv4_" + br, xu2)
        a3 = _cbr(sd, pre + "adjust3_%s.2" % br, _cbr(sd, pre + "adjust3_%s.1" % br, _cbr(sd, pre + "adjust3_%s.0" % br, x2)))
        a4 = _cbr(sd, pre + "adjust4_%s.1" % br, _cbr(sd, pre + "adjust4_%s.0" % br, x3))
        sm = F.conv2d(x4, sd[pre + "conv5_%s.weight" % br], sd[pre + "conv5_%s.bias" % br]) + _up(a3, 4) + _up(a4, 2)
        maps.append(sm)
    return maps


def soft_argmax(score_map, stride=4):
    """head.py:200-212 with coord grids :138-145 (x = stride * col, y = stride * row)."""
    B, _, H, W = score_map.shape
    idx = torch.arange(0, H).view(-1, 1) * stride
    coord_x = idx.repeat((H, 1)).view((H * W,)).float()
    coord_y = idx.repeat((1, H)).view((H * W,)).float()
    prob = F.softmax(score_map.view(-1, H * W), dim=1)
    return torch.sum(coord_x * prob, dim=1), torch.sum(coord_y * prob, dim=1)


def xyxy_to_cxcywh(b):
    x0, y0, x1, y1 = b.unbind(-1)
    return torch.stack([(x0 + x1) / 2, (y0 + y1) / 2, (x1 - x0), (y1 - y0)], dim=-1)


def cxcywh_to_xyxy(b):
    xc, yc, w, h = b.unbind(-1)
    return torch.stack([(xc - 0.5 * w), (yc - 0.5 * h), (xc + 0.5 * w), (yc + 0.5 * h)], dim=-1)


def corner_head(sd, pre, x):
    """Pyramid_Corner_Predictor.forward (head.py:147-157) -> (B,4) xyxy in [0,1]."""
    tl, br = corner_score_maps(sd, pre, x)
    img_sz = tl.shape[-1] * 4
    xtl, ytl = soft_argmax(tl)
    xbr, ybr = soft_argmax(br)
    return torch.stack((xtl, ytl, xbr, ybr), dim=1) / img_sz


# ----------------------------------------------------------------------------- score head
def score_decoder(sd, pre, search, template, box_xyxy, num_heads=12):
    """ScoreDecoder.forward, score_decoder.py:32-66 (PrRoIPool 4x4, scale 1.0)."""
    b, c, h, w = search.shape
    bb = (box_xyxy.clone() * w).view(-1, 4)
    rois = torch.cat([torch.arange(bb.shape[0], dtype=torch.float32).view(-1, 1), bb], 1)
    x = _ln(sd, pre + "norm1", sd[pre + "score_token"].expand(b, -1, -1), 1e-5)
    roi = torch.from_numpy(prroi_pool2d(search.detach().numpy(), rois.numpy(), 4, 4, 1.0))
    mem = [roi.flatten(2).transpose(1, 2), template.flatten(2).transpose(1, 2)]
    scale = c ** -0.5
    for i in range(2):
        q = _lin(sd, pre + "proj_q.%d" % i, x)
        k = _lin(sd, pre + "proj_k.%d" % i, mem[i])
        v = _lin(sd, pre + "proj_v.%d" % i, mem[i])
        q = q.view(b, -1, num_heads, c // num_heads).transpose(1, 2)
        k = k.view(b, -1, num_heads, c // num_heads).transpose(1, 2)
        v = v.view(b, -1, num_heads, c // num_heads).transpose(1, 2)
        a = F.softmax(torch.einsum("bhlk,bhtk->bhlt", q, k) * scale, dim=-1)
        x = torch.einsum("bhlt,bhtv->bhlv", a, v).transpose(1, 2).reshape(b, -1, c)
        x = _lin(sd, pre + "proj.%d" % i, x)
        x = _ln(sd, pre + "norm2.%d" % i, x, 1e-5)
    n = 0
    while (pre + "score_head.layers.%d.weight" % n) in sd:
        n += 1
    for i in range(n):
        x = _lin(sd, pre + "score_head.layers.%d" % i, x)
        if i < n - 1:
            x = F.relu(x)
    return x


# ----------------------------------------------------------------------------- models
@torch.no_grad()
def forward(sd, variant, template, online_template, search, run_score_head=False, return_aux=False, ce_forced=None,
            ce_template_mask=None):
    """Reference-equivalent forward.  template / online_template / search are [rgb, tir] lists
    of (B,3,H,W) fp32 CPU tensors.  Returns (out_dict, outputs_coord) like the reference;
    with return_aux also a dict of intermediates."""
    assert variant in VARIANTS, variant
    aux = {}
    if variant == "rgb":  # template / online_template / search: (B,3,H,W) tensors or [rgb] lists
        one = lambda x: x[0] if isinstance(x, (list, tuple)) else x  # noqa: E731
        _, _, sx = backbone_two_stream(sd, "backbone.", one(template), one(online_template), one(search))
        aux["search"] = sx
        tl, br = corner_score_maps(sd, "box_head.", sx)  # forward_box_head, mixformer.py:323-337
        aux["score_map_tl"], aux["score_map_br"] = tl, br
        img_sz = tl.shape[-1] * 4
        xtl, ytl = soft_argmax(tl)
        xbr, ybr = soft_argmax(br)
        xyxy = torch.stack((xtl, ytl, xbr, ybr), dim=1) / img_sz
        coord = xyxy_to_cxcywh(xyxy).view(sx.shape[0], 1, 4)
        out = {"pred_boxes": coord}
        return (out, coord, aux) if return_aux else (out, coord)
    if variant == "rgbt":
        tv, ov, sv = backbone_two_stream(sd, "backbone_v.", template[0], online_template[0], search[0])
        ti, oi, si = backbone_two_stream(sd, "backbone_i.", template[1], online_template[1], search[1])
        t_all = torch.cat([tv, ti], 0)
    else:
        fn = {"shared": backbone_shared, "asym_ce": backbone_asym_ce}.get(variant, backbone_asym)
        kw = ({"stages": aux.setdefault("ce_stages", []), "forced": ce_forced, "mask": ce_template_mask}
              if variant == "asym_ce" else {})
        t_all, _, s_all = fn(sd, "backbone.", torch.cat(template, 0), torch.cat(online_template, 0), torch.cat(search, 0),
                             **kw)
        Bh = s_all.shape[0] // 2
        sv, si = s_all[:Bh], s_all[Bh:]
    aux["search_v"], aux["search_i"] = sv, si
    fused = fusion_lnspecific(sd, "fusion_vi.", sv.contiguous(), si.contiguous())
    aux["fused"] = fused
    tl, br = corner_score_maps(sd, "box_head.", fused)
    aux["score_map_tl"], aux["score_map_br"] = tl, br
    img_sz = tl.shape[-1] * 4
    xtl, ytl = soft_argmax(tl)
    xbr, ybr = soft_argmax(br)
    xyxy = torch.stack((xtl, ytl, xbr, ybr), dim=1) / img_sz
    b = fused.shape[0]
    coord = xyxy_to_cxcywh(xyxy).view(b, 1, 4)
    out = {"pred_boxes": coord}
    if variant == "asym_online" and run_score_head:
        Bh = t_all.shape[0] // 2
        templ = torch.cat([t_all[:Bh], t_all[Bh:]], dim=2)
        aux["score_template"] = templ
        # forward_head, asymmetric_shared_online.py:405-410, called without gt_bboxes (:374): the ROI is
        # always the predicted box
        gt = cxcywh_to_xyxy(coord.clone().view(-1, 4))
        out["pred_scores"] = score_decoder(sd, "score_branch.", fused, templ, gt,
                                           num_heads=fused.shape[1] // 64).view(-1)
    if return_aux:
        return out, coord, aux
    return out, coord


def state_dict_to_torch(sd_np):
    return {k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in sd_np.items()}
