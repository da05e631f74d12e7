"""Synthetic stripe inputs of SURVEY.md §8(d): every stripe is uniform random
bytes from a counter-based generator, splitmix64 with base seed
0x5EED_0000 + config_id and stream = the GLOBAL stripe index, so a stripe's
bytes do not depend on how many GPUs share the job; plus fixed edge stripes
(all-0x00, all-0xFF, a 0..255 ramp) at global indices 0, 1, 2.

Stripe g's data bytes are the little-endian bytes of the words
    word(g, j) = mix64(seed_g + (j + 1) * GAMMA),  seed_g = mix64(base + (g + 1) * GAMMA)
for j = 0 .. k*L/8 - 1 over its k data rows laid end to end (row c holds
words [c*L/8, (c+1)*L/8)). `stripes_torch` builds them on the GPU with
wrapping int64 arithmetic; `stripe_numpy` is the uint64 CPU twin the tests
and bench checks use. Bench / test infrastructure, not product code.
"""
import numpy as np

GAMMA = 0x9E3779B97F4A7C15
C1 = 0xBF58476D1CE4E5B9
C2 = 0x94D049BB133111EB
EDGE_STRIPES = 3  # global stripes 0, 1, 2: all-0x00, all-0xFF, ramp


def base_seed(config_id):
    return 0x5EED0000 + int(config_id)


def _s64(x):
    """uint64 constant as the int64 with the same bits (torch has no uint64 math)."""
    x &= (1 << 64) - 1
    return x - (1 << 64) if x >= 1 << 63 else x


def mix64_numpy(z):
    z = np.asarray(z, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * np.uint64(C1)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(C2)
    return z ^ (z >> np.uint64(31))


def stripe_seed(config_id, g):
    with np.errstate(over="ignore"):
        return int(mix64_numpy(np.uint64(base_seed(config_id)) + np.uint64(g + 1) * np.uint64(GAMMA)))


def edge_row(g, L):
    if g == 0:
        return np.zeros(L, np.uint8)
    if g == 1:
        return np.full(L, 0xFF, np.uint8)
    return (np.arange(L) % 256).astype(np.uint8)


def stripe_numpy(config_id, g, k, L):
    """Data rows [k, L] of global stripe g (CPU reference of stripes_torch)."""
    if g < EDGE_STRIPES:
        return np.stack([edge_row(g, L)] * k)
    if L % 8:
        raise ValueError("cell bytes must be a multiple of 8")
    j = np.arange(1, k * L // 8 + 1, dtype=np.uint64)
    with np.errstate(over="ignore"):
        words = mix64_numpy(np.uint64(stripe_seed(config_id, g)) + j * np.uint64(GAMMA))
    return words.astype("<u8").view(np.uint8).reshape(k, L)


def _mix64_torch(torch, z):
    # logical right shifts of int64 bits: arithmetic shift, then mask the sign fill
    z = (z ^ ((z >> 30) & ((1 << 34) - 1))) * _s64(C1)
    z = (z ^ ((z >> 27) & ((1 << 37) - 1))) * _s64(C2)
    return z ^ ((z >> 31) & ((1 << 33) - 1))


def fill_data_rows(torch, stripes, config_id, g0, k, p, batch=8):
    """Writes the data rows (hops locations p..p+k-1) of stripes[S, k+p, L]
    (a CUDA uint8 tensor) for global stripes g0 .. g0+S-1; parity rows are
    left alone."""
    S, n, L = stripes.shape
    if n != k + p or L % 8:
        raise ValueError("stripes must be [S, k+p, L] with L % 8 == 0")
    W = k * L // 8
    j = torch.arange(1, W + 1, dtype=torch.int64, device=stripes.device) * _s64(GAMMA)  # wraps mod 2^64
    for s0 in range(0, S, batch):
        gs = list(range(g0 + s0, g0 + min(S, s0 + batch)))
        seeds = torch.tensor([_s64(stripe_seed(config_id, g)) for g in gs], dtype=torch.int64,
                             device=stripes.device)
        words = _mix64_torch(torch, seeds[:, None] + j[None, :])
        stripes[s0:s0 + len(gs), p:, :] = words.view(torch.uint8).view(len(gs), k, L)
        for i, g in enumerate(gs):
            if g < EDGE_STRIPES:
                stripes[s0 + i, p:, :] = torch.from_numpy(np.stack([edge_row(g, L)] * k)).to(stripes.device)
    return stripes
