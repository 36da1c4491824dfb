"""Deterministic synthetic weights and inputs ("mmt-synth-v1").

There are no trained checkpoints in this environment (the reference's are download-only,
README.md:9), so parity fixtures, tests and bench.py all use weights derived from a
counter-hash PRNG keyed by the state_dict name.  The same function produces the same bytes
here and on the GPU box, so no weight file is ever committed.

Generator: value(name, i) = 2 * u - 1 with u = top 24 bits of splitmix64(fnv1a64(name) ^ seed
+ (i + 1) * 0x9E3779B97F4A7C15) / 2**24, i.e. uniform on [-1, 1).  Each tensor is then scaled by
a rule chosen from its name/shape (unit-gain fan-in scaling for Linear/Conv weights, ~1 for
norm scales, small biases).  Two deliberate deviations from a plain init, both recorded in
SURVEY.md §7.1 / defect D8:
  * the corner-head output convolutions are amplified (HEAD_GAIN) so the 80x80 heat-maps are
    peaked and the soft-argmax box depends on the input (with default init every box is
    ~(0.49, 0.49, 0, 0) and box parity would be vacuous);
  * the fixed sin-cos position embeddings (pos_embed_s / pos_embed_t) get their real values
    (pos_utils.py:20-35 restated in `sincos_pos_embed`), as the reference computes them at init.
"""
from __future__ import annotations

import numpy as np

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)
GOLDEN = np.uint64(0x9E3779B97F4A7C15)

# Gain applied to the last convolution of every corner-head branch that produces a 1-channel
# score map (conv5_*, adjust3_*.2, adjust4_*.1).  Chosen so logits span ~+-10 (peaked maps).
HEAD_GAIN = 6.0


def fnv1a64(s: str) -> np.uint64:
    h = 0xCBF29CE484222325
    for b in s.encode():
        h ^= b
        h = (h * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF
    return np.uint64(h)


def _splitmix64(z: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = z + GOLDEN
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z


def uniform(name: str, shape, seed: int = 0) -> np.ndarray:
    """Counter-hash uniform [-1, 1) float32 tensor for `name`."""
    n = int(np.prod(shape)) if len(shape) else 1
    base = fnv1a64(name) ^ np.uint64(seed)
    with np.errstate(over="ignore"):
        ctr = base + (np.arange(n, dtype=np.uint64) + np.uint64(1)) * GOLDEN
    z = _splitmix64(ctr)
    u = (z >> np.uint64(40)).astype(np.float64) / float(1 << 24)
    return (2.0 * u - 1.0).astype(np.float32).reshape(shape)


def sincos_pos_embed(embed_dim: int, grid: int) -> np.ndarray:
    """2-D sin-cos table in fp64, cast to fp32 (pos_utils.py:20-66, mixformer.py:223-229).

    Note the reference's quirk: `np.meshgrid(grid_w, grid_h)` puts the *column* index in
    grid[0], and grid[0] feeds the first half of the channels."""
    gh = np.arange(grid, dtype=np.float64)
    gw = np.arange(grid, dtype=np.float64)
    g = np.stack(np.meshgrid(gw, gh), axis=0).reshape(2, 1, grid, grid)

    def one_d(d, pos):
        omega = np.arange(d // 2, dtype=np.float64) / (d / 2.0)
        omega = 1.0 / 10000 ** omega
        out = np.einsum("m,d->md", pos.reshape(-1), omega)
        return np.concatenate([np.sin(out), np.cos(out)], axis=1)

    emb = np.concatenate([one_d(embed_dim // 2, g[0]), one_d(embed_dim // 2, g[1])], axis=1)
    return emb.astype(np.float32)


def _is_head_output_conv(name: str) -> bool:
    return (
        (".conv5_tl." in name or ".conv5_br." in name or name.startswith("box_head.conv5_"))
        or ("adjust3_tl.2.0." in name or "adjust3_br.2.0." in name)
        or ("adjust4_tl.1.0." in name or "adjust4_br.1.0." in name)
    )


def synth_tensor(name: str, shape, seed: int = 0, grid_sizes=None) -> np.ndarray:
    """One state_dict entry of the synthetic model."""
    shape = tuple(int(s) for s in shape)
    if name.endswith("num_batches_tracked"):
        return np.zeros(shape, dtype=np.int64)
    if name.endswith("pos_embed_s") or name.endswith("pos_embed_t"):
        n, c = shape[-2], shape[-1]
        g = int(round(n ** 0.5))
        return sincos_pos_embed(c, g).reshape(shape)
    u = uniform(name, shape, seed)
    if name.endswith("running_mean"):
        return 0.1 * u
    if name.endswith("running_var"):
        return (1.0 + 0.25 * u).astype(np.float32)
    if name.endswith("level_embed"):
        return u * np.float32(np.sqrt(3.0))
    if name.endswith("score_token"):
        return 0.02 * u
    if "sampling_offsets" in name:
        if name.endswith("bias"):
            return 2.0 * u  # +-2 feature-map pixels (normaliser is 20)
        return u * np.float32(0.5 * np.sqrt(3.0 / shape[1]))
    if len(shape) == 1:
        if name.endswith("weight"):  # LayerNorm / GroupNorm / BatchNorm scale
            return (1.0 + 0.1 * u).astype(np.float32)
        return 0.02 * u  # any bias
    fan_in = int(np.prod(shape[1:]))
    w = u * np.float32(np.sqrt(3.0 / fan_in))
    if _is_head_output_conv(name) and name.endswith("weight"):
        w = w * np.float32(HEAD_GAIN)
    return w.astype(np.float32)


def synth_state_dict(keys_shapes, seed: int = 0):
    """{name: np.ndarray} for an ordered list of (name, shape)."""
    return {k: synth_tensor(k, s, seed) for k, s in keys_shapes}


def synth_inputs(batch: int, template_size: int = 128, search_size: int = 320, seed: int = 1):
    """Synthetic normalised frames, SURVEY §8(d): N(0,1) from torch.Generator().manual_seed(seed)
    drawn in the order t_v, t_i, o_v, o_i, s_v, s_i.  Returns CPU fp32 tensors."""
    import torch

    g = torch.Generator().manual_seed(seed)
    t = [torch.randn(batch, 3, template_size, template_size, generator=g) for _ in range(2)]
    o = [torch.randn(batch, 3, template_size, template_size, generator=g) for _ in range(2)]
    s = [torch.randn(batch, 3, search_size, search_size, generator=g) for _ in range(2)]
    return t, o, s
