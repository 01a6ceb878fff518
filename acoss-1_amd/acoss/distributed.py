"""Multi-GPU tiling of the N x N song-pair matrix.

One process per GPU (torch.distributed; backend "nccl" = RCCL over xGMI on ROCm, "gloo" on
CPU for tests). The pair matrix is split into contiguous ROW STRIPES whose cost
sum_i sum_j M'_i N'_j is balanced; every rank scores only its stripe (no data-path
collective), then ONE all-gather of the stripes assembles the full score matrix on every
rank — the exchange step that replaces the reference's shared np.memmap
(acoss/algorithms/algorithm_template.py:61,174-177).
"""
import numpy as np


def pair_cost(lens, i, j, m=9, tau=1):
    a = max(0, lens[i] - m * tau)
    b = max(0, lens[j] - m * tau)
    return float(a) * float(b)


def row_costs(lens, symmetric=True, m=9, tau=1):
    """Cost of each row of the pair matrix: upper triangle (symmetric) or full row."""
    s = np.maximum(np.asarray(lens, np.float64) - m * tau, 0)
    tot = s.sum()
    if symmetric:
        suffix = np.cumsum(s[::-1])[::-1]  # sum_{j >= i}
        after = suffix - s                 # sum_{j > i}
        return s * after
    return s * (tot - s)


def stripe_bounds(lens, world, symmetric=True, m=9, tau=1):
    """[(r0, r1)] per rank: contiguous rows with ~equal total cost."""
    c = row_costs(lens, symmetric, m, tau)
    n = len(c)
    cum = np.concatenate([[0.0], np.cumsum(c)])
    tot = cum[-1]
    cuts = [0]
    for r in range(1, world):
        cuts.append(int(np.searchsorted(cum, tot * r / world, side="left")))
    cuts.append(n)
    cuts = np.maximum.accumulate(np.clip(cuts, 0, n))
    return [(int(cuts[r]), int(cuts[r + 1])) for r in range(world)]


def stripe_pairs(n, r0, r1, symmetric=True):
    """(P, 2) int32 (query, reference) pairs of rows [r0, r1): j > i if symmetric else j != i."""
    out = []
    for i in range(r0, r1):
        js = np.arange(i + 1, n) if symmetric else np.concatenate([np.arange(0, i), np.arange(i + 1, n)])
        if len(js):
            out.append(np.stack([np.full(len(js), i), js], 1))
    return np.concatenate(out).astype(np.int32) if out else np.zeros((0, 2), np.int32)


def stripe_pair_chunks(n, r0, r1, symmetric=True, chunk=1 << 20):
    """The pairs of stripe_pairs(n, r0, r1, symmetric), same order, as (<= chunk, 2) int32 arrays,
    formed one chunk at a time (a Da-TACOS stripe holds 10^8 pairs: never materialised whole)."""
    buf, have = [], 0
    for i in range(r0, r1):
        js = np.arange(i + 1, n, dtype=np.int32) if symmetric else \
            np.concatenate([np.arange(0, i, dtype=np.int32), np.arange(i + 1, n, dtype=np.int32)])
        pos = 0
        while pos < len(js):
            take = min(chunk - have, len(js) - pos)
            part = np.empty((take, 2), np.int32)
            part[:, 0] = i
            part[:, 1] = js[pos:pos + take]
            buf.append(part)
            have += take
            pos += take
            if have == chunk:
                yield np.concatenate(buf) if len(buf) > 1 else buf[0]
                buf, have = [], 0
    if have:
        yield np.concatenate(buf) if len(buf) > 1 else buf[0]


def scatter_stripe(pairs, scores, r0, r1, n):
    """Local (r1-r0, n) block with the stripe's scores (zeros elsewhere, as the memmap)."""
    import torch
    blk = torch.zeros((r1 - r0, n), dtype=scores.dtype, device=scores.device)
    if len(pairs):
        p = pairs if isinstance(pairs, torch.Tensor) else torch.as_tensor(pairs)
        p = p.to(scores.device).long()
        blk[p[:, 0] - r0, p[:, 1]] = scores
    return blk


def all_gather_stripes(blk, bounds, group=None):
    """Assemble the full (n, n) matrix from every rank's row stripe (one all-gather)."""
    import torch
    import torch.distributed as dist
    n = blk.shape[1]
    rmax = max(r1 - r0 for r0, r1 in bounds)
    # gloo collectives take host tensors: route a device block through host memory
    host = dist.get_backend(group) == "gloo" and blk.is_cuda
    src = blk.cpu() if host else blk
    pad = torch.zeros((rmax, n), dtype=src.dtype, device=src.device)
    pad[: src.shape[0]] = src
    outs = [torch.empty_like(pad) for _ in bounds]
    dist.all_gather(outs, pad, group=group)
    full = torch.cat([o[: r1 - r0] for o, (r0, r1) in zip(outs, bounds)], 0)
    return full.to(blk.device) if host else full
