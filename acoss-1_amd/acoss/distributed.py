"""Multi-GPU tiling of the N x N song-pair matrix.

One process per GPU (torch.distributed; backend "nccl" = RCCL over xGMI on ROCm, "gloo" on
CPU for tests). The pair matrix is split into contiguous ROW STRIPES whose cost
sum_i sum_j M'_i N'_j is balanced; every rank scores only its stripe (no data-path
collective), then ONE exchange assembles the full score matrix — the step that replaces the
reference's shared np.memmap (acoss/algorithms/algorithm_template.py:61,174-177): an all-gather
onto every rank where every rank needs the matrices next (SNF late fusion, row-sharded), a gather
onto rank 0 where only rank 0 finishes, evaluates and saves them.
"""
import os

import numpy as np

# environment variables that name a process's rank on its node, in the order they are trusted
# (torch.distributed.run / torchrun, Open MPI, MPICH / Intel MPI, Slurm)
LOCAL_RANK_VARS = ("LOCAL_RANK", "OMPI_COMM_WORLD_LOCAL_RANK", "MPI_LOCALRANKID", "SLURM_LOCALID")


def local_rank(rank, n_dev):
    """This process's rank on its node: the launcher's variable, else rank % n_dev."""
    for v in LOCAL_RANK_VARS:
        s = os.environ.get(v)
        if s is not None and s.strip().lstrip("-").isdigit():
            return int(s)
    return rank % max(1, n_dev)


def bind_local_device():
    """One process per GPU: under the nccl (RCCL) backend bind this rank to GPU
    local_rank % device_count before the package allocates anything on "cuda".

    Without it every rank of `torchrun --nproc-per-node 8` that never called
    torch.cuda.set_device would allocate on cuda:0, and RCCL refuses (or serialises) several
    ranks on one GPU. The rule: a process whose current device is the default (cuda:0) is moved
    to its local rank's GPU; a process that already sits on its local rank's GPU, or that the
    caller bound to another non-default GPU on purpose, is left where it is. Under gloo (CPU
    collectives; ranks may share a GPU, as the tests do) nothing is bound. Returns the device
    index this rank uses under nccl, else None."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_backend() != "nccl":
        return None
    if not torch.cuda.is_available():
        return None
    n = torch.cuda.device_count()
    want = local_rank(dist.get_rank(), n) % n
    cur = torch.cuda.current_device()
    if cur != want and cur == 0:
        torch.cuda.set_device(want)
        cur = want
    return cur


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


def gather_stripes(blk, bounds, dst=0, group=None):
    """Assemble the full (n, n) matrix on rank `dst` only (one gather); other ranks get None.
    For scorers whose matrices only the root finishes, evaluates and saves (Serra09, SiMPle): no
    other rank receives, copies to host or writes the N x N matrix (0.9 GB per matrix at
    Da-TACOS size)."""
    import torch
    import torch.distributed as dist
    n = blk.shape[1]
    rmax = max(r1 - r0 for r0, r1 in bounds)
    host = dist.get_backend(group) == "gloo" and blk.is_cuda
    src = blk.cpu() if host else blk
    pad = torch.zeros((rmax, n), dtype=src.dtype, device=src.device)
    pad[: src.shape[0]] = src
    me = dist.get_rank(group)
    outs = [torch.empty_like(pad) for _ in bounds] if me == dst else None
    dist.gather(pad, gather_list=outs, dst=dst, group=group)
    if me != dst:
        return None
    full = torch.cat([o[: r1 - r0] for o, (r0, r1) in zip(outs, bounds)], 0)
    return full.to(blk.device) if host else full
