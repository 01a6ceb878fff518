/*
 * acoss_hip.h — C-ABI of libacoss_hip.so, the MI355X (gfx950) engine for the acoss
 * all-pairs cross-similarity + alignment hot path.
 *
 * Conventions:
 *  - Every array pointer is a DEVICE pointer owned by the caller (torch tensors), unless
 *    the parameter name ends in `_host`. Scalars are passed by value.
 *  - Row-major, C-contiguous. Chroma features are packed: track t occupies rows
 *    [track_off[t], track_off[t] + track_len[t]) of a (sum_len x 12) float32 block.
 *  - Every call is stream-ordered on `hip_stream` (a hipStream_t; NULL = default stream)
 *    and returns 0 on success or a negative ACOSS_E* code. No C++ exception crosses the
 *    ABI; acoss_last_error() returns a thread-local message for the last failure.
 *  - The only allocation is an internal, grow-only device workspace cache
 *    (acoss_release_workspace() frees it).
 *
 * Each entry point cites the reference interface it replaces (paths relative to the
 * reference repo silvadirceu/acoss-1).
 */
#ifndef ACOSS_HIP_H
#define ACOSS_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ACOSS_OK 0
#define ACOSS_E_ARG (-1)      /* invalid argument / unsupported parameter */
#define ACOSS_E_SHAPE (-2)    /* track too short for the frame stacking (n <= m*tau) */
#define ACOSS_E_HIP (-3)      /* HIP runtime error */
#define ACOSS_E_NONBINARY (-4)/* non-binary element in an alignment input (alignment_tools.py:22-23) */

/* Parameters of essentia ChromaCrossSimilarity + CoverSongSimilarity as acoss calls them
 * (acoss/algorithms/rqa_serra09.py:31-32,60-64; latefusion_chen.py:58-71). */
typedef struct acoss_crp_params {
  int32_t m;          /* frameStackSize, default 9 */
  int32_t tau;        /* frameStackStride, default 1 */
  float kappa;        /* binarizePercentile, default 0.095 */
  int32_t oti;        /* 1 = optimal transposition of the reference (default), 0 = none */
  float gamma_open;   /* disOnset, default 0.5 */
  float gamma_ext;    /* disExtension, default 0.5 */
} acoss_crp_params;

/* Library / build information. */
const char* acoss_version(void);
const char* acoss_last_error(void);
int acoss_release_workspace(void);

/* Optional phase timing (bench.py): HIP events recorded around every kernel launch on the
 * launch stream. enable(1) clears and starts recording, enable(0) stops. read() synchronises
 * the events and fills total_ms[i] / count[i] for phase i < n; returns the phase count.
 * Phase names: acoss_profile_phase_name(i). */
int acoss_profile_enable(int on);
int acoss_profile_read(double* total_ms, int64_t* count, int n);
const char* acoss_profile_phase_name(int i);

/* ---------------------------------------------------------------------------------
 * Serra09 / LateFusionChen hot path for a batch of song pairs (A1/A4/A9/A10/A16).
 * Replaces, per pair (i, j) = (pairs[2p], pairs[2p+1]):
 *   crp = essentia.ChromaCrossSimilarity(frameStackSize=m, frameStackStride=tau,
 *                                        binarizePercentile=kappa, oti=oti)(query, reference)
 *   _, qmax = essentia.CoverSongSimilarity('serra09', 'symmetric')(crp)
 *   _, dmax = essentia.CoverSongSimilarity('chen17',  'symmetric')(crp)
 * at acoss/algorithms/rqa_serra09.py:55-69 and acoss/algorithms/latefusion_chen.py:58-73.
 * query = track pairs[2p], reference = track pairs[2p+1]. qmax_out / dmax_out / oti_out are
 * float[n_pairs] / float[n_pairs] / int32[n_pairs] and each may be NULL (not computed).
 * max_len = max track_len over the tracks referenced (host scalar; sizes the workspace).
 * --------------------------------------------------------------------------------- */
int acoss_crp_align(const float* feats, const int64_t* track_off, const int32_t* track_len, int32_t n_tracks,
                    int32_t max_len, const int32_t* pairs, int64_t n_pairs, const acoss_crp_params* params,
                    float* qmax_out, float* dmax_out, int32_t* oti_out, void* hip_stream);

/* Single-pair CRP with every intermediate exposed (parity / debugging of A1/A4).
 * X: (M x 12), Y: (N x 12) device float32. Outputs (device, each may be NULL):
 *   dist (Mp x Np) float32 stacked Euclidean distances, thr_row (Mp), thr_col (Np) float32
 *   percentile thresholds, crp (Mp x Np) uint8 mutual-neighbour mask, oti (1) int32.
 * Mp = ceil((M - m*tau)/tau), Np likewise (essentia stackChromaFrames). */
int acoss_crp_pair(const float* X, int32_t M, const float* Y, int32_t N, const acoss_crp_params* params,
                   float* dist, float* thr_row, float* thr_col, uint8_t* crp, int32_t* oti, void* hip_stream);

/* essentia CoverSongSimilarity(alignmentType, distanceType='symmetric') on a given binary
 * matrix (A9/A10): crp (M x N) uint8 in {0,1}. align = 0 'serra09' (Qmax), 1 'chen17'
 * (dmax). score_out: float[1]. Replaces the alignment calls at rqa_serra09.py:64,67 and
 * latefusion_chen.py:67-71 when the CRP comes from elsewhere. */
int acoss_align_crp(const uint8_t* crp, int32_t M, int32_t N, int32_t align, float gamma_open, float gamma_ext,
                    float* score_out, void* hip_stream);

/* acoss smith_waterman_constrained (A8, acoss/algorithms/utils/alignment_tools.py:25-46) on
 * a batch of binary matrices: matrix b is (rows[b] x cols[b]) uint8 at byte offset off[b]
 * of `mats`. score_out: double[n_mats]. Bit-exact float64 (same evaluation order). */
int acoss_sw_constrained(const uint8_t* mats, const int64_t* off, const int32_t* rows, const int32_t* cols,
                         int32_t n_mats, int32_t max_rows, int32_t max_cols, double* score_out, void* hip_stream);

/* Cross-similarity matrices (A5/A6/A2): acoss get_csm / get_csm_cosine
 * (cross_recurrence.py:30-73), optionally after get_csm_blocked_oti's query rotation
 * (:105-134): with oti_shift >= 0 every 12-bin block of each X row is rolled by oti_shift
 * (np.roll on the chroma axis) first. X (M x d), Y (N x d) float32; out (M x N) float32.
 * kind = 0 euclidean, 1 cosine, 2 self-similarity of X (get_ssm :10-28; Y ignored). */
int acoss_csm(const float* X, int32_t M, const float* Y, int32_t N, int32_t d, int32_t kind, int32_t oti_shift,
              float* out, void* hip_stream);

/* acoss get_oti (cross_recurrence.py:75-103) for a batch: C1, C2 (n x 12) float32 global
 * chroma vectors; out int32[n] = argmax_i sum(roll(C1[k], i) * C2[k]), first max wins. */
int acoss_get_oti(const float* C1, const float* C2, int32_t n, int32_t* out, void* hip_stream);

/* acoss csm_to_binary (A7, cross_recurrence.py:136-161): row-wise kappa nearest neighbours.
 * D (M x N) float32 -> B (M x N) uint8. nneighbs = number of ones per row (the host computes
 * int(np.round(kappa * N)) or kappa itself, as the reference does); nneighbs <= 0 -> all ones.
 * Among equal distances the lowest column index wins (numpy's argpartition choice is
 * arbitrary). */
int acoss_binarize_rows(const float* D, int32_t M, int32_t N, int32_t nneighbs, uint8_t* B, void* hip_stream);

/* acoss getWCSM (A14, similarity_fusion.py:38-54): W = exp(-CSM^2 / (2 (mu*Eps)^2)) with
 * Eps = (rowmean_k2 + colmean_k1 + CSM)/3 of the k2 / k1 smallest per row / column.
 * CSM, W: (M x N) float32. The means add the k smallest in ascending order and exp is the
 * canonical canon_expf, so W equals the CPU oracle's (oracle/ef_oracle.cpp or_ef_wcsm) bit for bit. */
int acoss_wcsm(const float* CSM, int32_t M, int32_t N, int32_t k1, int32_t k2, float mu, float* W,
               void* hip_stream);

/* out[i] = exp(-x[i]) for n float32 values, in the canonical float32 exp shared with the CPU oracle
 * (common.hpp canon_expf): EarlyFusion's early matrix np.exp(-WCSM_sum)
 * (earlyfusion_traile.py:182) for the per-pair path (EarlyFusion.pair_matrices); the batched
 * acoss_earlyfusion applies the same exp inside. out may alias x. */
int acoss_neg_exp(const float* x, int64_t n, float* out, void* hip_stream);

/* One cross-diffusion step of similarity network fusion for matrix `skip` (f2, replaces the body
 * of the loop at acoss/algorithms/utils/similarity_fusion.py:163-174 in doSimilarityFusionWs):
 *   out = S . A . S^T + reg_diag * I,  A = (sum_{m != skip} mats[m]) / (n_mats - 1),
 * S the kNN-truncated row-normalised affinity (getS, :121-143) given as J (n x K) int32 column
 * indices and V (n x K) float64 values, any order within a row (sums run in ascending column
 * order, as scipy's csr product). Every J entry must lie in [0, n) and no column may repeat
 * within a row (scipy's coo -> csr would merge repeats into one term): otherwise ACOSS_E_ARG,
 * checked on the device before any product runs. mats: HOST array of n_mats device pointers
 * to (n x n) float64 matrices; out (n x n) float64 may alias mats[skip] but no other.
 * n_mats >= 2 (any number; more than 16 others are averaged in passes), 0 < K <= min(n, 64).
 * validate = 1: the index check synchronises the stream once and a bad J returns ACOSS_E_ARG;
 * validate = 0 (J already checked, e.g. once per fusion): no sync, and a bad row is replaced by
 * a weight-0 entry on its own column, so no kernel reads outside the matrices. */
int acoss_snf_step(const double* const* mats, int32_t n_mats, int32_t skip, int32_t n, const int32_t* J,
                   const double* V, int32_t K, double reg_diag, double* out, int32_t validate, void* hip_stream);

/* The same step split at its one exchange point, for a fusion row-sharded across ranks (SURVEY
 * §8f row 2: each rank owns rows [row0, row0 + rows) of every matrix; the same loop body,
 * similarity_fusion.py:163-174). Both halves are bit-identical to the matching rows of
 * acoss_snf_step: same kernels, same summation order.
 *   acoss_snf_diffuse_rows: B_rows = rows [row0, row0 + rows) of B = A . S^T, from the (rows x n)
 *     stripes mats[m] of the matrices (HOST array of device pointers); B_rows (rows x n) may
 *     overlap mats[skip] but no other stripe.
 *   (the caller all-gathers the stripes of B into the whole (n x n) B)
 *   acoss_snf_left_rows: out = rows [row0, row0 + rows) of S . B + reg_diag * I, from the whole
 *     (n x n) B; out (rows x n) must not overlap B.
 * J, V, K, validate as for acoss_snf_step (J, V describe all n rows of S in both calls). */
int acoss_snf_diffuse_rows(const double* const* mats, int32_t n_mats, int32_t skip, int32_t n, int32_t rows,
                           const int32_t* J, const double* V, int32_t K, double* B_rows, int32_t validate,
                           void* hip_stream);
int acoss_snf_left_rows(const double* B, int32_t n, int32_t row0, int32_t rows, const int32_t* J, const double* V,
                        int32_t K, double reg_diag, double* out, int32_t validate, void* hip_stream);

/* SiMPle matrix profile score (A11, acoss/algorithms/simple_silva.py:68-118) for a batch of
 * ordered pairs, including the per-pair OTI roll of the reference (Simple.oti, :45-54).
 * feats: packed (12 x n_t) float64 blocks, track t at element offset track_off[t] (dim-major,
 * as the reference's seq arrays). score_out[p] = median_i min_j dist (the reference stores
 * -score, simple_silva.py:125). apply_oti = 0 scores the reference as given (Simple.simple_sim
 * alone); oti_out (may be NULL) always receives the Simple.oti index. */
int acoss_simple_mp(const double* feats, const int64_t* track_off, const int32_t* track_len, int32_t n_tracks,
                    int32_t max_len, const int32_t* pairs, int64_t n_pairs, int32_t sslen, int32_t apply_oti,
                    double* score_out, int32_t* oti_out, void* hip_stream);

/* Per-track median downsampling of chroma (A13: Serra09/ChenFusion.load_features,
 * acoss/algorithms/rqa_serra09.py:44-53 and latefusion_chen.py:46-56, which call
 * librosa.util.sync(chroma.T, arange(0, n, factor), aggregate=np.median)).
 * feats: packed (sum n, 12) float32, track t at frame offset track_off[t]; max_len = max n.
 * out: track t's ceil(n_t / factor) x 12 float32 rows at frame offset out_off[t].
 * factor <= 64. */
int acoss_median_downsample(const float* feats, const int64_t* track_off, const int32_t* track_len, int32_t n_tracks,
                            int32_t max_len, int32_t factor, float* out, const int64_t* out_off, void* hip_stream);

/* Per-track SiMPle features (A12: Simple.load_features + Simple.smooth,
 * acoss/algorithms/simple_silva.py:34-43,56-66): window means (win=200, hop skip=100) ->
 * 'same' zero-filled convolution with the host weights smooth[0..smooth_len) (normalised
 * symmetric Hann(6) in the reference) -> per-column L2 normalisation.
 * out: track t's (12 x floor(n_t / skip)) float64 block (dim-major) at element offset
 * out_off[t]; out_elems = total doubles in out. smooth is a HOST pointer. */
int acoss_simple_features(const float* feats, const int64_t* track_off, const int32_t* track_len, int32_t n_tracks,
                          int32_t win, int32_t skip, const double* smooth, int32_t smooth_len, double* out,
                          const int64_t* out_off, int64_t out_elems, void* hip_stream);

/* Batched EarlyFusion scores (A15: EarlyFusion.similarity, acoss/algorithms/earlyfusion_traile.py:157-198).
 * Block features of every track packed row-major: mfcc (sum nb x d_mfcc), ssm (sum nb x d_ssm),
 * chroma (sum nb x d_chroma, 12-bin blocks) float32, track t's rows at block_off[t], n_blocks[t]
 * of them; chroma_med (n_tracks x 12) float32. For every pair: CSMs (euclid, euclid, blocked-OTI
 * cosine), csm_to_binary(kappa), getWCSM(K, K, mu) fusion, and smith_waterman_constrained of the
 * four binary matrices -> scores_out[4 p + {0: mfccs, 1: ssms, 2: chromas, 3: early}] (float64).
 * Pairs are processed in the order given; for large lists, order them (reference band, query) as
 * acoss/_lib.py earlyfusion does (1.24x at 15,000 Da-TACOS-shaped songs): a band of reference
 * tracks' rows then stays cached while the query rows stream past. */
int acoss_earlyfusion(const float* mfcc, const float* ssm, const float* chroma, const float* chroma_med,
                      const int64_t* block_off, const int32_t* n_blocks, int32_t n_tracks, int32_t max_blocks,
                      int32_t d_mfcc, int32_t d_ssm, int32_t d_chroma, const int32_t* pairs, int64_t n_pairs,
                      double kappa, int32_t K, float mu, double* scores_out, void* hip_stream);

/* EarlyFusion beat-synchronous block features of a batch of tracks (replaces
 * EarlyFusion.load_features' block loops, acoss/algorithms/earlyfusion_traile.py:67-154, and its
 * skimage resize_block, :214-247, restated in float64). Track t: chroma frames [frame_off[t],
 * +n_frames[t]) of chroma ((sum n) x 12) and MFCC frames [mfcc_off[t], +mfcc_frames[t]) of mfcc
 * ((sum n_mfcc) x d_mfcc, frame-major: mfcc_htk transposed, NaN already zeroed; the extractor's
 * mfcc_htk has fewer frames than the chroma, features.py:884); onsets (frame indices, int64) at
 * [onset_off[t], ...), its n_blocks = n_onsets - blocksize blocks at global block index
 * block_off[t] .. (total_blocks in all). Block b spans mfcc[o[b] : o[b+blocksize-1]] and
 * chroma[o[b] : o[b+blocksize]], each clamped to its own frame count as Python slicing does
 * (resize_block's X[i1:i2], :240); the caller guarantees every clamped span is non-empty (the
 * reference raises on an empty one). Outputs per global block: out_mfcc (mfccs_per_block *
 * d_mfcc), out_ssm (mfccs_per_block (mfccs_per_block - 1) / 2), out_chroma (chromas_per_block *
 * 12) float32; out_med (n_tracks x 12) = np.median(chroma, axis=0). */
int acoss_ef_block_features(const float* mfcc, const float* chroma, const int64_t* frame_off, const int32_t* n_frames,
                            const int64_t* mfcc_off, const int32_t* mfcc_frames,
                            const int64_t* onsets, const int64_t* onset_off, const int64_t* block_off,
                            int32_t n_tracks, int64_t total_blocks, int32_t blocksize, int32_t mfccs_per_block,
                            int32_t chromas_per_block, int32_t d_mfcc, float* out_mfcc, float* out_ssm,
                            float* out_chroma, float* out_med, void* hip_stream);

/* Finish of a pair-score matrix after the pair loop, in place when out == D.
 * D, out: (n x n) float32, row stride ld (elements). symmetric = 1 first forms D[i,j] + D[j,i] from
 * the original values (CoverAlgorithm.all_pairwise's `Ds += Ds.T`, algorithm_template.py:188-191);
 * mode 0 stops there, 1 divides by norm[j] (Serra09.normalize_by_length, rqa_serra09.py:71-83),
 * 2 stores norm[j] / D (ChenFusion.normalize_by_length, latefusion_chen.py:75-85); norm: float64[n]
 * = sqrt(frames of song j), the quotient taken in float64 and rounded to float32 as the
 * reference's float32 memmap does. */
int acoss_ds_finish(const float* D, int32_t n, int64_t ld, const double* norm, int32_t symmetric, int32_t mode,
                    float* out, void* hip_stream);

/* The rank step of CoverAlgorithm.getEvalStatistics (algorithm_template.py:206-291): for query q
 * (song q_song[q]) and each song j = members[m_off[q] .. m_off[q+1]), ranks_out[that index] = the
 * 1-based position of j in np.argsort(-D', 1, kind="stable") of the query's row, where D' is D
 * with the diagonal set to -inf (:234) and columns ordered by pos[] (each song's position in the
 * reference's clique ordering, :220-230; NaN scores sort last). D: (n x n) float32, stride ld. */
int acoss_eval_ranks(const float* D, int32_t n, int64_t ld, const int32_t* pos, const int32_t* q_song,
                     const int64_t* m_off, const int32_t* members, int32_t n_queries, int32_t* ranks_out,
                     void* hip_stream);

/* ---------------------------------------------------------------------------------
 * Per-track feature files (.npz twins of the reference's deepdish .h5 files), read on native
 * threads: replaces the per-song `dd.io.load` of CoverAlgorithm.load_features
 * (acoss/algorithms/algorithm_template.py:90) and EarlyFusion.load_features
 * (acoss/algorithms/earlyfusion_traile.py:88-99) for a whole batch of songs in two calls.
 * Host only (no GPU); every pointer is a HOST pointer. */
typedef struct acoss_npz_member {
  int32_t file;        /* index into paths */
  int32_t method;      /* zip method: 0 stored (np.savez), 8 deflate (np.savez_compressed) */
  int32_t ndim;
  int32_t fortran;     /* fortran_order of the .npy header */
  int64_t shape[8];
  int64_t nbytes;      /* bytes of array data (itemsize * prod(shape)) */
  int64_t member_off;  /* file offset of the member (the .npy stream) */
  int64_t comp_size;   /* its compressed size */
  int64_t npy_size;    /* its uncompressed size */
  int64_t data_skip;   /* offset of the array data inside the .npy stream */
  char name[128];      /* member name without ".npy", e.g. "madmom_features/onsets" */
  char descr[32];      /* numpy dtype descr, e.g. "<f4", "<U6" (object dtypes are refused) */
} acoss_npz_member;

/* Index n_files npz files: every member whose top-level key (the name up to the first '/') is
 * one of `keys_host` ('\n'-separated; NULL = every member), in file order, then zip order.
 * *n_out = the member count; ACOSS_E_ARG (message names the file) on an unreadable file or when
 * the count exceeds max_out (retry with *n_out). n_threads <= 0: every hardware thread. */
int acoss_npz_index(const char* const* paths_host, int32_t n_files, const char* keys_host, int32_t n_threads,
                    acoss_npz_member* out_host, int64_t max_out, int64_t* n_out);

/* Read every member's array data into dst_host[i] (nbytes each), one thread per file. */
int acoss_npz_read(const char* const* paths_host, const acoss_npz_member* members_host, int64_t n_members,
                   void* const* dst_host, int32_t n_threads);

#ifdef __cplusplus
}
#endif
#endif /* ACOSS_HIP_H */
