"""Similarity network fusion (acoss/algorithms/utils/similarity_fusion.py) on the GPU.

Same functions and arguments as the reference; numpy in, numpy out, device tensors inside.
`getWCSM` runs the HIP kernel (misc.hip); each cross-diffusion step S . P . S^T runs as the HIP
kernels of snf.hip (acoss_snf_step: two row-sparse products, O(N^2 K), not a dense N^3 GEMM,
summed in scipy's csr order). W, P and the kNN sets (torch.topk) are one-off device tensor ops.

Two reference behaviours are kept on purpose:
  * dtypes follow numpy's: float32 inputs give float32 W/P, the diffusion runs in float64;
  * in doSimilarityFusionWs, `Pts = nextPts` aliases the two lists after the first
    iteration, so from the second iteration on every update of matrix i already sees the
    updated matrices k < i (similarity_fusion.py:157-177). The loop below is written the
    same way, so it has the same aliasing.
The kNN choices among exactly tied values are unspecified in both (np.argpartition / topk).
"""
import numpy as np

from ... import _lib

__all__ = ["getW", "getWCSM", "setupWCSMSSM", "getWCSMSSM", "getP", "getS", "doSimilarityFusionWs",
           "doSimilarityFusion"]


def _t(x, dtype=None):
    torch = _lib._torch()
    if isinstance(x, torch.Tensor):
        t = x.cuda()
    else:
        a = np.asarray(x)
        t = torch.as_tensor(np.ascontiguousarray(a)).cuda()
    return t.to(dtype) if dtype is not None else t


def _np(t):
    return t.detach().cpu().numpy()


def _getW(D, K, Mu=0.5):
    torch = _lib._torch()
    DSym = 0.5 * (D + D.T)
    DSym.fill_diagonal_(0)
    Neighbs = torch.topk(DSym, K + 1, dim=1, largest=False).values
    # the reference's order: (mean * (K + 1)) / K, in the input dtype (similarity_fusion.py:27)
    MeanDist = Neighbs.mean(1) * float(K + 1) / float(K)
    Eps = (MeanDist[:, None] + MeanDist[None, :] + DSym) / 3
    Denom = 2 * (Mu * Eps) ** 2
    Denom[Denom == 0] = 1
    return torch.exp(-DSym ** 2 / Denom)


def getW(D, K, Mu=0.5):
    """Affinity matrix (similarity_fusion.py:15-36)."""
    return _np(_getW(_t(D), K, Mu))


def getWCSM(CSMAB, k1, k2, Mu=0.5):
    """Cross-similarity affinity (similarity_fusion.py:38-54), HIP kernel."""
    return _np(_lib.wcsm(np.asarray(CSMAB, np.float32), k1, k2, Mu))


def setupWCSMSSM(WSSMA, WSSMB, WCSMAB):
    """[[WSSMA, WCSMAB], [WCSMAB^T, WSSMB]] (similarity_fusion.py:56-74)."""
    M, N = WSSMA.shape[0], WSSMB.shape[0]
    W = np.zeros((N + M, N + M))
    W[:M, :M] = WSSMA
    W[:M, M:] = WCSMAB
    W[M:, :M] = WCSMAB.T
    W[M:, M:] = WSSMB
    return W


def getWCSMSSM(SSMA, SSMB, CSMAB, K, Mu=0.5):
    """Parent W with the neighbours split between SSM and CSM parts (similarity_fusion.py:76-96)."""
    M, N = SSMA.shape[0], SSMB.shape[0]
    k1 = int(K * float(M) / (M + N))
    k2 = K - k1
    return setupWCSMSSM(getW(SSMA, k1, Mu), getW(SSMB, k2, Mu), getWCSM(CSMAB, k1, k2, Mu))


def _getP(W, diagRegularize=False):
    torch = _lib._torch()
    if diagRegularize:
        WNoDiag = W.clone()
        WNoDiag.fill_diagonal_(0)
        RowSum = WNoDiag.sum(1)
        RowSum[RowSum == 0] = 1
        eye = torch.eye(W.shape[0], dtype=torch.float64, device=W.device)
        return 0.5 * eye + 0.5 * WNoDiag / RowSum[:, None]
    RowSum = W.sum(1)
    RowSum[RowSum == 0] = 1
    return W / RowSum[:, None]


def getP(W, diagRegularize=False):
    """Row-normalised probability matrix (similarity_fusion.py:98-119)."""
    return _np(_getP(_t(W), diagRegularize))


class _KNN:
    """Row-sparse matrix with K entries per row: S[i, J[i, k]] = V[i, k]."""

    def __init__(self, J, V, n):
        self.J, self.V, self.n = J, V, n

    def todense(self):
        torch = _lib._torch()
        S = torch.zeros((self.n, self.n), dtype=self.V.dtype, device=self.V.device)
        S.scatter_(1, self.J, self.V)
        return S


def _getS(W, K):
    torch = _lib._torch()
    V, J = torch.topk(W, K, dim=1, largest=True)
    SNorm = V.sum(1)
    SNorm[SNorm == 0] = 1
    return _KNN(J, V / SNorm[:, None], W.shape[0])


def getS(W, K):
    """kNN-truncated, row-normalised W (similarity_fusion.py:121-143), as a scipy CSR matrix."""
    from scipy import sparse
    S = _getS(_t(W), K)
    J, V = _np(S.J), _np(S.V)
    n = W.shape[0]
    return sparse.coo_matrix((V.ravel(), (np.repeat(np.arange(n), J.shape[1]), J.ravel())), shape=(n, n)).tocsr()


def _fusion_ws(Ws, K=5, niters=20, reg_diag=1):
    torch = _lib._torch()
    Ps = [_getP(W) for W in Ws]
    Ss = [_getS(W, K) for W in Ws]
    # float32 P upcast once (exact): in the reference the first iteration adds the float32 Ps
    # into float64 accumulators, every later one adds float64 matrices
    Pts = [P.to(torch.float64).contiguous() for P in Ps]
    N = len(Pts)
    if N < 2:
        if N == 0:
            raise IndexError("list index out of range")  # the reference's Ws[0] (similarity_fusion.py:167)
        if niters > 0:
            # the reference divides the empty sum by float(N - 1) = 0 (similarity_fusion.py:176):
            # 0/0 = nan everywhere, which every later step keeps
            import warnings
            warnings.warn("invalid value encountered in divide", RuntimeWarning, stacklevel=3)
            return torch.full(Pts[0].shape, float("nan"), dtype=torch.float64, device=Pts[0].device)
        return Pts[0].clone()
    # each S is fixed across the iterations: its kNN columns are checked once here, and the
    # steps skip the per-step check (and the stream sync it costs)
    Js = [S.J.to(torch.int32).contiguous() for S in Ss]
    Vs = [S.V.to(torch.float64).contiguous() for S in Ss]
    for Jt in Js:
        _lib.check_knn(Jt, Pts[0].shape[0])
    world, rank = _shard_world()
    if world > 1 and Pts[0].shape[0] >= world:  # (fewer rows than ranks: every rank runs it whole)
        plan = shard_plan(Pts, Js, Vs, reg_diag, world, rank)
        if plan["shard"]:
            return _fusion_sharded(Pts, Js, Vs, niters, reg_diag, world, rank)
    for it in range(niters):
        # the reference's `Pts = nextPts` aliasing: from the second iteration on, matrix i's
        # update already sees the new matrices k < i; replacing Pts[i] in place of the list
        # entry reproduces that, and the first iteration (separate lists) sees only old ones
        nxt = list(Pts) if it == 0 else Pts
        for i in range(N):
            nxt[i] = _lib.snf_step(Pts, i, Js[i], Vs[i], reg_diag, validated=True)
        Pts = nxt
    Fused = torch.zeros(Pts[0].shape, dtype=torch.float64, device=Pts[0].device)
    for Pt in Pts:
        Fused += Pt
    return Fused / N


def _shard_world():
    """(world, rank) of the torch.distributed job when the fusion may row-shard across its ranks,
    else (1, 0). ACOSS_SNF_SHARD=0 keeps every rank on the whole matrices (replicated)."""
    import os
    import torch.distributed as dist
    if os.environ.get("ACOSS_SNF_SHARD", "auto") == "0":
        return 1, 0
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        return dist.get_world_size(), dist.get_rank()
    return 1, 0


# the last sharding decision (shard_plan), for logs and the bench line
LAST_PLAN = {}


def shard_plan(Pts, Js, Vs, reg_diag, world, rank, force=None, repeats=2):
    """Decide row-sharded vs replicated cross-diffusion by measurement, the same way on every rank.

    A replicated step for one matrix costs t_rep on every rank. Sharded, a rank computes its 1/W
    of the rows of both halves (about t_rep / W) and waits for ONE all-gather of B (n x n float64,
    the exchange) per step. Both grow as n^2, so the choice depends on the exchange bandwidth
    against HBM, not on n: sharding pays when t_gather < t_rep (1 - 1/W). This times one
    replicated step (result discarded) and one all-gather of B-sized stripes, takes the maximum
    over ranks, and shards when t_gather <= 0.8 t_rep (1 - 1/W) (20 % margin for the per-step
    launch and synchronisation costs the estimate leaves out). Each time is the minimum of
    `repeats` runs after one untimed warm-up of each operation (first-launch module loads and
    first-use buffer registration are not the steady state). ACOSS_SNF_SHARD=1 forces sharding
    without measuring; an explicit force=True/False from the caller still measures and reports the
    rule, then applies `force`; =0 never reaches here; the default is this rule ("auto")."""
    import os
    import time
    import torch.distributed as dist
    from ... import distributed as _dist
    torch = _lib._torch()
    mode = os.environ.get("ACOSS_SNF_SHARD", "auto")
    n = int(Pts[0].shape[0])
    if force is None and mode == "1":
        LAST_PLAN.clear()
        LAST_PLAN.update({"n": n, "world": world, "backend": dist.get_backend(), "mode": mode,
                          "t_step_replicated_ms": None, "t_gather_B_ms": None, "gather_GBps": None,
                          "rule_shard": None, "shard": True})
        return dict(LAST_PLAN)
    bounds = shard_rows(n, world)
    r0, r1 = bounds[rank]

    def sync():
        if Pts[0].is_cuda:
            torch.cuda.synchronize()

    def timed(fn):
        fn()  # warm-up
        best = float("inf")
        for _ in range(repeats):
            dist.barrier()
            sync()
            t0 = time.perf_counter()
            fn()
            sync()
            best = min(best, time.perf_counter() - t0)
        return best
    t_rep = timed(lambda: _lib.snf_step(Pts, 0, Js[0], Vs[0], reg_diag, validated=True))
    Bs = torch.zeros((r1 - r0, n), dtype=torch.float64, device=Pts[0].device)
    t_gather = timed(lambda: _dist.all_gather_stripes(Bs, bounds))
    del Bs
    on_dev = dist.get_backend() == "nccl"
    t = torch.tensor([t_rep, t_gather], dtype=torch.float64, device="cuda" if on_dev else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    t_rep, t_gather = float(t[0]), float(t[1])
    rule = t_gather <= 0.8 * t_rep * (1.0 - 1.0 / world)
    shard = bool(force) if force is not None else rule
    LAST_PLAN.clear()
    LAST_PLAN.update({"n": n, "world": world, "backend": dist.get_backend(), "mode": mode,
                      "t_step_replicated_ms": round(t_rep * 1e3, 3), "t_gather_B_ms": round(t_gather * 1e3, 3),
                      "gather_GBps": round(8.0 * n * n * (world - 1) / world / max(t_gather, 1e-9) / 1e9, 1),
                      "rule_shard": bool(rule), "shard": shard})
    return dict(LAST_PLAN)


def shard_rows(n, world):
    """[(r0, r1)] per rank: row stripes within one row of each other (every row of a step costs the
    same, K gathered rows); none is empty when n >= world."""
    return [(r * n // world, (r + 1) * n // world) for r in range(world)]


def _fusion_sharded(Pts, Js, Vs, niters, reg_diag, world, rank):
    """The cross-diffusion loop row-sharded across ranks. Rank r owns rows
    [r0, r1) of every Pts[i]. A step for matrix i needs B = A . S^T whole but A only by rows:
    B's rows a come from A's rows a (acoss_snf_diffuse_rows), the stripes of B are all-gathered
    (the one exchange per step), and each rank forms its rows of S . B (acoss_snf_left_rows).
    The loop order, the `Pts = nextPts` aliasing and every sum are those of the replicated loop,
    so the gathered result is bit-identical to it."""
    from ... import distributed as _dist
    torch = _lib._torch()
    n = Pts[0].shape[0]
    bounds = shard_rows(n, world)
    r0, r1 = bounds[rank]
    St = [P[r0:r1].contiguous() for P in Pts]
    N = len(St)
    for it in range(niters):
        nxt = list(St) if it == 0 else St
        for i in range(N):
            Bs = _lib.snf_diffuse_rows(St, i, n, Js[i], Vs[i], validated=True)
            B = _dist.all_gather_stripes(Bs, bounds)
            nxt[i] = _lib.snf_left_rows(B, r0, r1 - r0, Js[i], Vs[i], reg_diag, validated=True)
            del B
        St = nxt
    Fused = torch.zeros_like(St[0])
    for Pt in St:
        Fused += Pt
    Fused = Fused / N
    return _dist.all_gather_stripes(Fused, bounds)


def doSimilarityFusionWs(Ws, K=5, niters=20, reg_diag=1):
    """Cross-diffusion of affinity matrices (similarity_fusion.py:145-182)."""
    return _np(_fusion_ws([_t(W) for W in Ws], K, niters, reg_diag))


def doSimilarityFusion(Scores, K=5, niters=5, reg_diag=1):
    """(list of W, fused similarity) from N x N distance matrices (similarity_fusion.py:184-192)."""
    Ws = [_getW(_t(D), K) for D in Scores]
    fused = _fusion_ws(Ws, K, niters, reg_diag)
    return [_np(W) for W in Ws], _np(fused)
