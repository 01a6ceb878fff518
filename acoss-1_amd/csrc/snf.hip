// Similarity network fusion, cross-diffusion step (f2; acoss/algorithms/utils/similarity_fusion.py:146-186).
//
// One step of doSimilarityFusionWs for matrix i:
//   A   = (sum_{m != i} Pts[m]) / (L - 1)                    (similarity_fusion.py:165-169)
//   out = S_i . ((S_i . A^T)^T) + reg_diag * I                 (:171-174)
// with S_i the kNN-truncated, row-normalised W_i (getS, :121-143): K entries per row.
// (S A^T)^T = A S^T, so the step is two row-sparse products, both as COALESCED row gathers:
//   At        = A^T                            (k_snf_avg_t: the average, transposed via LDS)
//   B         = (S . At)^T                     (k_snf_spmm<true>: B^T[j, :] = sum_k V[j,k] At[J[j,k], :],
//                                               written transposed through an LDS tile)
//   out[i, :] = sum_k V[i,k] * B[J[i,k], :]    (k_snf_spmm<false>)
// so B[a, j] = sum_k V[j,k] * A[a, J[j,k]], the reference's inner product, term for term.
// Both products sum over k in ascending column order from 0, one rounded multiply and one
// rounded add per term (-ffp-contract=off), as scipy's csr_matvecs does on the csr matrix that
// getS builds (coo -> csr sorts the column indices); the transposes are exact, and the average
// is formed in the reference's order (m ascending, then one division). All float64.
//
// Traffic per step (n x n float64 each): the transpose reads the L-1 other matrices and writes
// At; each gather reads K row segments per output row (from the L2 working set of its column
// chunk, see k_snf_spmm) and writes one matrix. Algorithmic HBM bytes: (L - 1 + 1 + 2 + 2) * 8 * n^2 = (L + 4) * 8 n^2.
#include "common.hpp"

namespace acoss {
namespace {

// The matrices to average reach the kernel as kernel-argument chunks of kSnfChunk pointers;
// more than one chunk is summed in passes through a scratch matrix (same summation order).
constexpr int kSnfChunk = 16;
constexpr int kSnfMaxK = 64;

struct MatPtrs {
  const double* p[kSnfChunk];
};

// Per row: the K (column, value) pairs sorted by column (insertion sort; K <= 64), so both
// products sum in csr order. A row whose columns leave [0, n) or repeat (scipy's coo -> csr
// would merge repeats into one term) raises *err and is replaced by one harmless entry
// (its own column, weight 0), so no later kernel reads outside the matrices.
__global__ void k_snf_sort_knn(const int32_t* __restrict__ J, const double* __restrict__ V, int32_t n, int32_t K,
                               int32_t* __restrict__ Js, double* __restrict__ Vs, int32_t* __restrict__ err) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  int32_t jj[kSnfMaxK];
  double vv[kSnfMaxK];
  for (int k = 0; k < K; ++k) {
    int32_t c = J[(int64_t)r * K + k];
    double v = V[(int64_t)r * K + k];
    int q = k;
    while (q > 0 && jj[q - 1] > c) {
      jj[q] = jj[q - 1];
      vv[q] = vv[q - 1];
      --q;
    }
    jj[q] = c;
    vv[q] = v;
  }
  bool ok = jj[0] >= 0 && jj[K - 1] < n;
  for (int k = 1; k < K; ++k) ok = ok && jj[k] != jj[k - 1];
  if (!ok) {
    *err = 1;
    for (int k = 0; k < K; ++k) {
      jj[k] = r;
      vv[k] = 0.0;
    }
  }
  for (int k = 0; k < K; ++k) {
    Js[(int64_t)r * K + k] = jj[k];
    Vs[(int64_t)r * K + k] = vv[k];
  }
}

// At[c, a] = (sum_{m != skip} mats[m][a, c]) / (n_mats - 1): 64 x 64 tile through LDS, over the
// `rows` rows a of a row stripe (the mats are (rows, n) stripes; At is (n, rows)).
// One launch sums a chunk of `cnt` matrices (the skipped one already left out, ascending m)
// onto the running sum `part` (untransposed; NULL for the first chunk). A chunk that is not
// the last writes the running sum to `part_out` untransposed; the last divides and writes At.
// A middle chunk reads and writes the same running sum (part == part_out): each element is read
// and then written by the same thread, and the two pointers are not __restrict__.
__global__ __launch_bounds__(256) void k_snf_avg_t(MatPtrs mats, int32_t cnt, int32_t rows, int32_t n, double denom,
                                                   const double* part, double* part_out,
                                                   double* __restrict__ At) {
  __shared__ double tile[64][65];
  const int a0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
  const int t = threadIdx.x;
#pragma unroll 4
  for (int r = 0; r < 16; ++r) {
    const int idx = t + 256 * r;
    const int a = a0 + (idx >> 6), c = c0 + (idx & 63);
    double s = 0.0;
    if (a < rows && c < n) {
      const int64_t e = (int64_t)a * n + c;
      if (part) s = part[e];
      for (int m = 0; m < cnt; ++m) s = s + mats.p[m][e];
      if (part_out)
        part_out[e] = s;
      else
        s = s / denom;
    }
    tile[idx & 63][idx >> 6] = s;
  }
  if (part_out) return;  // uniform per launch
  __syncthreads();
#pragma unroll 4
  for (int r = 0; r < 16; ++r) {
    const int idx = t + 256 * r;
    const int c = c0 + (idx >> 6), a = a0 + (idx & 63);
    if (a < rows && c < n) At[(int64_t)c * rows + a] = tile[idx >> 6][idx & 63];
  }
}

// Both products are row gathers of a dense matrix D by the sparse S (K entries per row):
//   R[r, c] = sum_k Vs[r,k] * D[Js[r,k], c]   (ascending k, one rounded multiply and add per term)
// TRANS (gather): D = At (n x rows), r = j in [0, n), written transposed as B[c, j];
// !TRANS (left):  D = B (n x n), r = i in [row0, row0 + rows), written as out[i - row0, c]
//                 (+ reg_diag on the diagonal, after the sum, as the reference's separate
//                 `nextPts[i][pix, pix] += reg_diag`).
// Tiling for the caches: a block is kSnfRB output rows x kSnfW columns of D, and the blocks are
// ordered column-chunk-major per XCD (xcd_remap): each XCD walks its own run of chunks, every
// output row of a chunk before the next, so the K gathered segments of all rows come from that
// XCD's L2 working set, D[:, chunk] = n x kSnfW doubles (3.8 MB at n = 15,000), instead of
// the whole of D (1.8 GB, which the first versions gathered from at 4-7 TB/s of HBM/MALL).
constexpr int kSnfW = 32;   // columns per chunk
constexpr int kSnfRB = 32;  // output rows per block
// VW consecutive columns per lane (VW = 2: 16-byte gathers, 16 lanes per row segment, when the
// row pitch and the column count are even); 256 / (kSnfW / VW) row groups per pass.
template <bool TRANS, int VW>
__global__ __launch_bounds__(256) void k_snf_spmm(const double* __restrict__ D, int64_t ldd, int32_t dcols,
                                                  int32_t nout, int32_t row0, int32_t K,
                                                  const int32_t* __restrict__ Js, const double* __restrict__ Vs,
                                                  double reg_diag, double* __restrict__ out, int64_t ldo,
                                                  int32_t rblocks) {
  constexpr int LPR = kSnfW / VW, RG = 256 / LPR;  // lanes per row segment, row groups
  typedef double dvec __attribute__((ext_vector_type(VW)));
  __shared__ double tile[TRANS ? kSnfW : 1][kSnfRB + 1];
  __shared__ int32_t sj[kSnfRB * kSnfMaxK];
  __shared__ double sv[kSnfRB * kSnfMaxK];
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  const int chunk = L / rblocks, rb = L - chunk * rblocks;
  const int cl = (threadIdx.x % LPR) * VW, rg = threadIdx.x / LPR;
  const int c = chunk * kSnfW + cl;
  const bool cok = c < dcols;  // VW = 2: dcols is even, so c + 1 < dcols too
  // the block's kNN rows (contiguous in Js/Vs) staged in LDS: the gathers below then issue
  // without a dependent index load in front of each
  const int r0 = rb * kSnfRB, nr = min(kSnfRB, nout - r0);
  for (int t = threadIdx.x; t < nr * K; t += 256) {
    sj[t] = Js[(int64_t)(row0 + r0) * K + t];
    sv[t] = Vs[(int64_t)(row0 + r0) * K + t];
  }
  __syncthreads();
  const dvec* Dc = reinterpret_cast<const dvec*>(D + (cok ? c : 0));
  const int64_t ldv = ldd / VW;
#pragma unroll
  for (int q = 0; q < kSnfRB / RG; ++q) {
    const int rl = rg + RG * q;
    const int r = r0 + rl;  // output row (0-based within the output)
    dvec acc = 0.0;
    if (rl < nr) {
      const int i = row0 + r;  // kNN row
      const int32_t* jr = sj + rl * K;
      const double* vr = sv + rl * K;
      int k = 0;
      for (; k + 4 <= K; k += 4) {  // four gathers in flight, summed in k order
        const dvec x0 = Dc[jr[k] * ldv], x1 = Dc[jr[k + 1] * ldv];
        const dvec x2 = Dc[jr[k + 2] * ldv], x3 = Dc[jr[k + 3] * ldv];
        acc = acc + vr[k] * x0;
        acc = acc + vr[k + 1] * x1;
        acc = acc + vr[k + 2] * x2;
        acc = acc + vr[k + 3] * x3;
      }
      for (; k < K; ++k) acc = acc + vr[k] * Dc[jr[k] * ldv];
      if (!TRANS && cok) {
#pragma unroll
        for (int v = 0; v < VW; ++v)
          if (c + v == i && reg_diag > 0.0) acc[v] = acc[v] + reg_diag;
        *reinterpret_cast<dvec*>(out + (int64_t)r * ldo + c) = acc;
      }
    }
    if (TRANS) {
#pragma unroll
      for (int v = 0; v < VW; ++v) tile[cl + v][rl] = acc[v];
    }
  }
  if constexpr (TRANS) {
    __syncthreads();
    // B[c, r]: kSnfW runs of kSnfRB consecutive doubles
#pragma unroll
    for (int t = 0; t < (kSnfW * kSnfRB) / 256; ++t) {
      const int idx = threadIdx.x + 256 * t;
      const int cc = idx / kSnfRB, rr = idx % kSnfRB;
      const int oc = chunk * kSnfW + cc, orow = rb * kSnfRB + rr;
      if (oc < dcols && orow < nout) out[(int64_t)oc * ldo + orow] = tile[cc][rr];
    }
  }
}

// Launch of k_snf_spmm over nout output rows and dcols columns of D.
template <bool TRANS>
int snf_spmm(const double* D, int64_t ldd, int32_t dcols, int32_t nout, int32_t row0, int32_t K, const int32_t* Js,
             const double* Vs, double reg_diag, double* out, int64_t ldo, hipStream_t s) {
  const int32_t rblocks = (nout + kSnfRB - 1) / kSnfRB, nchunks = (dcols + kSnfW - 1) / kSnfW;
  const char* vwenv = getenv("ACOSS_SNF_VW");
  const bool even = ldd % 2 == 0 && dcols % 2 == 0 && reinterpret_cast<uintptr_t>(D) % 16 == 0 &&
                    (TRANS || (ldo % 2 == 0 && reinterpret_cast<uintptr_t>(out) % 16 == 0));
  const bool v2 = even && !(vwenv && vwenv[0] == '1');
  auto kern = v2 ? k_snf_spmm<TRANS, 2> : k_snf_spmm<TRANS, 1>;
  hipLaunchKernelGGL(kern, dim3((unsigned)rblocks * (unsigned)nchunks), dim3(256), 0, s, D, ldd, dcols, nout, row0, K,
                     Js, Vs, reg_diag, out, ldo, rblocks);
  ACOSS_LAUNCH_CHECK();
  return ACOSS_OK;
}

}  // namespace
}  // namespace acoss

using namespace acoss;

namespace {

bool snf_args_ok(const int32_t* J, const double* V, int32_t n, int32_t K) {
  return n > 0 && J && V && K > 0 && K <= kSnfMaxK && K <= n;
}

// Sorts the kNN rows into csr order (Js, Vs in workspace slot 12, after `lead` bytes) and, with
// `validate`, checks them (one stream sync) before any product reads a row they name. Without it
// a bad row has already been made harmless (its own column, weight 0), so no kernel reads
// outside the matrices; a caller that validated J once per fusion skips the sync.
int snf_sorted_knn(const int32_t* J, const double* V, int32_t n, int32_t K, int32_t validate, size_t lead,
                   hipStream_t s, char** ws_out, int32_t** Js, double** Vs) {
  const size_t knn = align_up((size_t)n * K, 64);
  char* ws = static_cast<char*>(workspace(12, lead + knn * 12 + 512));
  if (!ws) return ACOSS_E_HIP;
  *Vs = reinterpret_cast<double*>(ws + lead);
  *Js = reinterpret_cast<int32_t*>(ws + lead + knn * 8);
  int32_t* d_err = reinterpret_cast<int32_t*>(ws + lead + knn * 12);
  ACOSS_HIP_CHECK(hipMemsetAsync(d_err, 0, 4, s));
  hipLaunchKernelGGL(k_snf_sort_knn, dim3((n + 255) / 256), dim3(256), 0, s, J, V, n, K, *Js, *Vs, d_err);
  ACOSS_LAUNCH_CHECK();
  if (validate) {
    int h_err = 0;
    ACOSS_HIP_CHECK(hipMemcpyAsync(&h_err, d_err, 4, hipMemcpyDeviceToHost, s));
    ACOSS_HIP_CHECK(hipStreamSynchronize(s));
    if (h_err) {
      set_error("acoss_snf: kNN column indices must lie in [0, %d) without repeats within a row", n);
      return ACOSS_E_ARG;
    }
  }
  *ws_out = ws;
  return ACOSS_OK;
}

// B = (S . At)^T over a (rows, n) row stripe of the average of the other matrices: the average
// in the reference's order (m ascending, chunks of kSnfChunk pointers, one division), its
// transpose At (n x rows), then the gather. A multi-chunk running sum lives in B (free until
// the gather writes it).
int snf_diffuse(const double* const* mats, int32_t n_mats, int32_t skip, int32_t n, int32_t rows,
                const int32_t* Js, const double* Vs, int32_t K, double* At, double* B, hipStream_t s) {
  const double denom = (double)(n_mats - 1);
  const unsigned nc = (unsigned)((n + 63) / 64), nr = (unsigned)((rows + 63) / 64);
  MatPtrs mp{};
  int cnt = 0, done = 0;
  const double* part = nullptr;
  for (int m = 0; m < n_mats; ++m) {
    if (m == skip) continue;
    mp.p[cnt++] = mats[m];
    ++done;
    if (cnt == kSnfChunk || done == n_mats - 1) {
      const bool last = done == n_mats - 1;
      hipLaunchKernelGGL(k_snf_avg_t, dim3(nc, nr), dim3(256), 0, s, mp, cnt, rows, n, denom, part,
                         last ? nullptr : B, At);
      ACOSS_LAUNCH_CHECK();
      part = B;
      cnt = 0;
    }
  }
  // B[a, j] = sum_k Vs[j,k] * At[Js[j,k], a]: rows j of S over the stripe's columns a of At
  return snf_spmm<true>(At, rows, rows, n, 0, K, Js, Vs, 0.0, B, n, s);
}

bool overlaps(const double* a, size_t na, const double* b, size_t nb) {
  return a < b + nb && b < a + na;
}

}  // namespace

extern "C" int acoss_snf_step(const double* const* mats, int32_t n_mats, int32_t skip, int32_t n,
                              const int32_t* J, const double* V, int32_t K, double reg_diag, double* out,
                              int32_t validate, void* hip_stream) {
  clear_error();
  if (!mats || n_mats < 2 || skip < 0 || skip >= n_mats || !out || !snf_args_ok(J, V, n, K)) {
    set_error("acoss_snf_step: bad arguments (need n_mats >= 2, 0 <= skip < n_mats, 0 < K <= min(n, %d))",
              kSnfMaxK);
    return ACOSS_E_ARG;
  }
  for (int m = 0; m < n_mats; ++m) {
    if (!mats[m] || (m != skip && mats[m] == out)) {
      set_error("acoss_snf_step: matrix %d is NULL or aliases the output", m);
      return ACOSS_E_ARG;
    }
  }
  hipStream_t s = static_cast<hipStream_t>(hip_stream);
  const size_t nn = (size_t)n * n;
  char* ws = nullptr;
  int32_t* Js = nullptr;
  double* Vs = nullptr;
  int rc = snf_sorted_knn(J, V, n, K, validate, 2 * nn * 8, s, &ws, &Js, &Vs);
  if (rc != ACOSS_OK) return rc;
  double* Bm = reinterpret_cast<double*>(ws);
  double* At = reinterpret_cast<double*>(ws + nn * 8);
  rc = snf_diffuse(mats, n_mats, skip, n, n, Js, Vs, K, At, Bm, s);
  if (rc != ACOSS_OK) return rc;
  return snf_spmm<false>(Bm, n, n, n, 0, K, Js, Vs, reg_diag, out, n, s);
}

extern "C" int acoss_snf_diffuse_rows(const double* const* mats, int32_t n_mats, int32_t skip, int32_t n,
                                      int32_t rows, const int32_t* J, const double* V, int32_t K, double* B_rows,
                                      int32_t validate, void* hip_stream) {
  clear_error();
  if (!mats || n_mats < 2 || skip < 0 || skip >= n_mats || rows <= 0 || rows > n || !B_rows ||
      !snf_args_ok(J, V, n, K)) {
    set_error("acoss_snf_diffuse_rows: bad arguments (need n_mats >= 2, 0 <= skip < n_mats, 0 < rows <= n, "
              "0 < K <= min(n, %d))", kSnfMaxK);
    return ACOSS_E_ARG;
  }
  const size_t sn = (size_t)rows * n;
  for (int m = 0; m < n_mats; ++m) {
    if (!mats[m] || (m != skip && overlaps(mats[m], sn, B_rows, sn))) {
      set_error("acoss_snf_diffuse_rows: stripe %d is NULL or overlaps the output", m);
      return ACOSS_E_ARG;
    }
  }
  hipStream_t s = static_cast<hipStream_t>(hip_stream);
  char* ws = nullptr;
  int32_t* Js = nullptr;
  double* Vs = nullptr;
  int rc = snf_sorted_knn(J, V, n, K, validate, sn * 8, s, &ws, &Js, &Vs);
  if (rc != ACOSS_OK) return rc;
  return snf_diffuse(mats, n_mats, skip, n, rows, Js, Vs, K, reinterpret_cast<double*>(ws), B_rows, s);
}

extern "C" int acoss_snf_left_rows(const double* B, int32_t n, int32_t row0, int32_t rows, const int32_t* J,
                                   const double* V, int32_t K, double reg_diag, double* out, int32_t validate,
                                   void* hip_stream) {
  clear_error();
  if (!B || !out || row0 < 0 || rows <= 0 || rows > n - row0 || !snf_args_ok(J, V, n, K)) {
    set_error("acoss_snf_left_rows: bad arguments (need 0 <= row0, 0 < rows <= n - row0, 0 < K <= min(n, %d))",
              kSnfMaxK);
    return ACOSS_E_ARG;
  }
  if (overlaps(B, (size_t)n * n, out, (size_t)rows * n)) {
    set_error("acoss_snf_left_rows: the output overlaps B");
    return ACOSS_E_ARG;
  }
  hipStream_t s = static_cast<hipStream_t>(hip_stream);
  char* ws = nullptr;
  int32_t* Js = nullptr;
  double* Vs = nullptr;
  int rc = snf_sorted_knn(J, V, n, K, validate, 0, s, &ws, &Js, &Vs);
  if (rc != ACOSS_OK) return rc;
  return snf_spmm<false>(B, n, n, rows, row0, K, Js, Vs, reg_diag, out, n, s);
}
