/*
 * spectralmc_hip.h — C ABI of the MI355X (gfx950) GbmCVNNPricer hot path.
 *
 * One shared library, libspectralmc_hip.so, exports these symbols with plain
 * pointers and sizes (no torch / HIP C++ types in the signatures).  Every entry
 * point is stream-ordered on the caller's `hipStream_t` (passed as `void*`,
 * NULL = legacy default stream), allocates nothing per call, performs no host
 * synchronisation and no hidden H2D/D2H copy, so a caller may capture any
 * sequence of these calls into a hipGraph.  All device buffers are caller-owned.
 *
 * Reference seams replaced (Tuee22/SpectralMC @ 2026-01-02, paths relative to
 * the reference repository root):
 *   smc_sobol_*          scipy.stats.qmc.Sobol(d, scramble=True, seed) + fast_forward + random,
 *                        as used by SobolSampler.create / sample
 *                        (src/spectralmc/sobol_sampler.py:177-203, 222-246)
 *   smc_gbm_simulate     ConcurrentNormGenerator.get_matrix + SimulateBlackScholes[grid, tpb, stream]
 *                        (src/spectralmc/async_normals.py:388-398, src/spectralmc/gbm.py:224-257, 400-426)
 *   smc_gbm_normalize    forward normalisation sims *= forwards / row_means
 *                        (src/spectralmc/gbm.py:428-440)
 *   smc_cf_targets       put payoff + reshape(M, N) + FFT(axis=1) + mean(axis=0)
 *                        (src/spectralmc/gbm.py:464-474, src/spectralmc/gbm_trainer.py:806-817)
 *   smc_train_targets    the fused per-step Monte-Carlo side of _run_batch: all of the above for
 *                        B contracts in one launch sequence (src/spectralmc/gbm_trainer.py:1546-1556)
 *   smc_normals          the normal matrix the engine consumes for contract ordinal m
 *                        (async_normals.py:212-216 stream semantics; values are this library's RNG)
 *
 * Status codes are mapped to the reference's error dataclasses by the Python
 * host layer (spectralmc_amd/_lib.py); smc_last_error_string() gives the text of
 * the last failure on the calling thread.
 */
#ifndef SPECTRALMC_HIP_H
#define SPECTRALMC_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SMC_ABI_VERSION 15  /* 14: smc_time_launches; 15: SMC_MATH_REF | SMC_MATH_HW */

/* ---- status codes ------------------------------------------------------- */
#define SMC_OK                      0
#define SMC_ERR_INVALID_ARGUMENT    1  /* null pointer, bad enum, dim out of range    */
#define SMC_ERR_INVALID_SHAPE       2  /* sizes the kernels cannot take (e.g. N>4096)  */
#define SMC_ERR_SEED_OUT_OF_RANGE   3  /* seed/skip outside what the engine accepts    */
#define SMC_ERR_SEQUENCE_EXHAUSTED  4  /* Sobol index would pass 2^30 points           */
#define SMC_ERR_MEMORY_LIMIT        5  /* reference gbm.py:106-137 path-count guard     */
#define SMC_ERR_HIP                 6  /* HIP runtime error (launch / device)           */
#define SMC_ERR_EXCHANGE_TIMEOUT    7  /* a co-resident partner workgroup never arrived
                                          (smc_sync_status; NaN targets were written)     */

/* ---- enums (values mirror the reference enums' order) ------------------- */
#define SMC_SCHEME_LOG_EULER     0  /* PathScheme.LOG_EULER   effects/montecarlo.py:24-29 */
#define SMC_SCHEME_SIMPLE_EULER  1  /* PathScheme.SIMPLE_EULER                           */
#define SMC_NORM_RAW             0  /* ForwardNormalization.RAW  effects/montecarlo.py:30-35 */
#define SMC_NORM_NORMALIZE       1  /* ForwardNormalization.NORMALIZE                    */
#define SMC_DTYPE_F32            0  /* Precision.float32 (paths f32, targets complex64)  */
#define SMC_DTYPE_F64            1  /* Precision.float64 (paths f64, targets complex128) */
#define SMC_MATH_HW          0x100  /* flag, OR into `scheme` (engine calls) or `dtype` (smc_normals):
                                      f32 hardware transcendentals (v_exp/v_log/v_sin/v_cos/v_sqrt)
                                      instead of the portable, CPU-reproducible kernels */
#define SMC_MATH_REF         0x400  /* flag, OR into smc_train_targets' / smc_train_step's `scheme` (f32
                                      only): the reference kernel's own typing (gbm.py:224-257 under
                                      Numba: f64 state and step of the f32 normals, f32 stores): portable
                                      normals, the f64 engine's step, rounded f32 paths (rows_ref_kernel +
                                      cf_kernel).  The f64 step's exp is within 2 ulp of libm's, so a
                                      stored f32 value equals the reference arithmetic's except where the
                                      two exps round to different floats (C2 shape: <= 1e-6 of the values,
                                      1 ulp; tests/test_oracle.py).  With SMC_MATH_HW (ABI 15): the same
                                      step on the hardware-transcendental f32 normals (~1 ulp from the
                                      portable ones, so not bit-reproducible on a CPU).  In the kernel
                                      queries' dtype: that kernel's name */
#define SMC_TRAIN_DYNAMIC    0x200  /* flag, OR into smc_train_step's `scheme`: the whole-contract resident
                                      launch hands out every contract from its contract queue (default:
                                      the first three quarters of the rounds statically), for launches that
                                      may start while the previous step's launch still holds CUs */
#define SMC_STORE_TERMINAL       1  /* keep only the terminal row [B][P] (scratch)        */
#define SMC_STORE_ALL            2  /* materialise the full path matrix [B][T][P]         */

#define SMC_SOBOL_BITS 30           /* scipy Sobol bits=30: at most 2^30 points          */

typedef struct smc_sobol smc_sobol;

int32_t     smc_abi_version(void);
const char* smc_last_error_string(void);
/* Kernel timing for measurement (ABI 14): arms two caller-created hipEvent_t for the engine calls that
 * follow on this thread (smc_train_step, smc_train_targets, smc_basket_train_targets): their first path /
 * CF kernel records start_event at its own start, every path / CF kernel records stop_event at its own
 * end (hipExtLaunchKernel), so after the call the pair spans the call's path and CF kernels as a kernel
 * trace times them, without the dispatch gaps of stream events around back-to-back launches.  The
 * auxiliary kernels (Sobol draw, cursor update, normalisation, normals) are not timed.  NULL, NULL
 * disarms.  Stream-ordered like the launches; captured launches record nothing. */
int32_t     smc_time_launches(void* start_event, void* stop_event);

/* ---- sync-area status (smc_train_step, smc_basket_train_targets) ---------- */
/* Launches whose workgroups exchange sums (the sliced resident kernel, the resident basket kernel)
 * poll for their partners a bounded time (~1 s).  A partner that never arrives (e.g. the group's
 * workgroups were not all co-resident) sets SMC_SYNC_EXCHANGE_TIMEOUT in the 32-bit status word at
 * byte SMC_SYNC_STATUS_OFFSET of the sync area and the launch's own failure flag (byte
 * SMC_SYNC_LAUNCH_FAIL_OFFSET); the launch still completes (every later wait of THAT launch sees its
 * flag and gives up at once) with NaN targets for the contracts it could not finish.  The last
 * workgroup of the launch clears the flag, so the next launch waits normally; the status word is
 * sticky across launches: the caller reads (and clears) it with smc_sync_status. */
#define SMC_SYNC_STATUS_OFFSET     32
#define SMC_SYNC_LAUNCH_FAIL_OFFSET 48
#define SMC_SYNC_EXCHANGE_TIMEOUT  1u
/* Waits for `stream`, then copies the status word of sync_dev to *status_out (0: no failure) and,
 * if clear != 0, zeroes it.  The only call of this ABI that synchronises the host. */
int32_t smc_sync_status(void* sync_dev, int32_t clear, int32_t* status_out, void* stream);
/* ---- scrambled Sobol (SciPy-bit-exact) ---------------------------------- */
/* Build the LMS+digital-shift scrambled generator SciPy builds for
 * Sobol(d=dim, scramble=True, seed=seed), then fast_forward(skip).
 * dim in [1, 64]; seed in [0, 2^63). */
int32_t smc_sobol_create(int32_t dim, uint64_t seed, uint64_t skip, smc_sobol** out);
void    smc_sobol_destroy(smc_sobol* h);
/* Host copies of the scrambled tables and the host cursor (next point index). */
int32_t smc_sobol_state(const smc_sobol* h, uint32_t* shift /*[dim]*/, uint32_t* sv /*[dim*30]*/,
                        uint64_t* cursor);
int32_t smc_sobol_fast_forward(smc_sobol* h, uint64_t n);
/* Host draw of n raw points in [0,1) (Sobol.random(n)); advances the host cursor. */
int32_t smc_sobol_random_host(smc_sobol* h, int64_t n, double* out /*[n][dim] host*/);
/* Table image for the device draw: tables[0..dim) = shift, tables[dim + d*30 + c] = sv[d][c].
 * The caller copies it into a device buffer of dim*31 u32 it owns. */
int32_t smc_sobol_export_tables(const smc_sobol* h, uint32_t* tables /*[dim*31] host*/);
/* Device draw from an uploaded table image: point i of the batch is sequence index
 *   (*index_dev if index_dev != NULL else 0) + index0 + i
 * scaled as lower + (upper - lower) * x in f64 exactly as sobol_sampler.py:239.
 * out_f64: [n][dim] f64 (required); out_f32: [n][dim] f32 copy or NULL (CVNN input,
 * gbm_trainer.py:1775-1783).  The caller guarantees the index range stays < 2^30. */
int32_t smc_sobol_draw(const uint32_t* tables_dev, int32_t dim, const int64_t* index_dev,
                       int64_t index0, int64_t n, const double* lower_dev, const double* upper_dev,
                       double* out_f64, float* out_f32, void* stream);

/* ---- GBM Monte-Carlo engine --------------------------------------------- */
/* contracts_dev: [B][6] f64 rows in BlackScholes.Inputs order X0, K, T, r, d, v.
 * Contract b uses normal stream ordinal (*ordinal_dev if non-NULL else 0) + ordinal0 + b.
 * paths_dev: [B][T][P] of the dtype (raw, un-normalised paths; row t = value after step t+1).
 * rowsum_dev: [B][T] f64 sums over the P paths of each row (may be NULL). */
int32_t smc_gbm_simulate(const double* contracts_dev, int64_t n_contracts, int32_t timesteps,
                         int64_t n_paths, uint64_t mc_seed, const int64_t* ordinal_dev,
                         int64_t ordinal0, int32_t scheme, int32_t dtype,
                         void* paths_dev, double* rowsum_dev, void* stream);
/* In-place forward normalisation of a [B][T][P] path matrix from its row sums. */
int32_t smc_gbm_normalize(const double* contracts_dev, int64_t n_contracts, int32_t timesteps,
                          int64_t n_paths, int32_t dtype, void* paths_dev,
                          const double* rowsum_dev, void* stream);
/* CF targets from a stored raw path matrix ([B][T][P], row T-1 is read) and its
 * row sums: targets[b][k] = FFT_N(mean_M(put.reshape(M, N)))[k], N*M == P. */
int32_t smc_cf_targets(const double* contracts_dev, int64_t n_contracts, int32_t timesteps,
                       int32_t network_size, int32_t batches_per_mc_run, int32_t normalization,
                       int32_t dtype, const void* paths_dev, const double* rowsum_dev,
                       void* targets_dev, void* stream);
/* Fused training targets: simulate + (store) + normalise + payoff + M-mean + DFT for
 * B contracts.  store_mode SMC_STORE_ALL writes the full matrix into paths_dev, which
 * holds `chunk_contracts` contracts ([chunk][T][pitch]) and is reused chunk by chunk;
 * SMC_STORE_TERMINAL needs paths_dev of [chunk][pitch].  path_pitch: elements between
 * consecutive path rows (0 = P, contiguous; else a multiple of 4 >= P, e.g. smc_path_pitch).
 * targets_dev: [B][N] complex.
 * workspace_dev (may be NULL): smc_engine_workspace_bytes(chunk, T, P, rowsum_dev != NULL)
 * bytes, zero-filled once before first use (the kernel leaves it zeroed).  With a workspace
 * each contract is simulated by several workgroups (slices of 8192 paths) and the last one
 * to finish runs the payoff/DFT phase; without it one workgroup runs the whole contract.
 * Results are bit-identical run to run either way; the two differ only in the f64 row-sum
 * association (oracle/gbm_oracle.c restates both). */
int32_t smc_train_targets(const double* contracts_dev, int64_t n_contracts, int32_t timesteps,
                          int32_t network_size, int32_t batches_per_mc_run, uint64_t mc_seed,
                          const int64_t* ordinal_dev, int64_t ordinal0, int32_t scheme,
                          int32_t normalization, int32_t dtype, int32_t store_mode,
                          void* paths_dev, int64_t path_pitch, int64_t chunk_contracts,
                          double* rowsum_dev, void* targets_dev, void* workspace_dev,
                          int64_t workspace_bytes, void* stream);
/* One Monte-Carlo step of the training loop (sobol_sampler.py:222-246 + gbm_trainer.py:1546-1556):
 * the Sobol draw of the step's contracts (point i = sequence index cursor_dev[0] + index_offset + i,
 * scaled as smc_sobol_draw, into contracts_dev [B][6] f64 and cvnn_input_dev [B][6] f32 or NULL),
 * the targets with ordinal_dev = cursor_dev + 1, ordinal0 = index_offset, then
 * cursor_dev[0..1] += advance.  Where the resident kernel takes the shape (f32, T = 16, P a
 * multiple of 4096 up to 8 x 65,536, N | 4096) each chunk of contracts is ONE launch: each
 * workgroup draws the rows of its own contracts and the last workgroup of the last chunk advances
 * the cursor.  P <= 65,536: one workgroup per contract, targets bit-identical to
 * smc_sobol_draw + smc_train_targets (no workspace) + the cursor update.  P > 65,536 (C3): W =
 * P / 65,536 co-resident workgroups per contract exchange their terminal and column sums through
 * the sync area; the f64 sums are added in slice order (oracle kernel mode, slices = W).  Other
 * shapes run the three steps as separate launches, bit-identical to the separate calls.
 * sync_dev: smc_train_step_sync_bytes(...) bytes, zero-filled before the first call (every call
 * leaves its counters zeroed; the status word at SMC_SYNC_STATUS_OFFSET is sticky, see
 * smc_sync_status). */
int32_t smc_train_step(const uint32_t* sobol_tables_dev, int32_t dim, const double* lower_dev,
                       const double* upper_dev, int64_t* cursor_dev, int64_t index_offset, int64_t advance,
                       double* contracts_dev, float* cvnn_input_dev, int64_t n_contracts, int32_t timesteps,
                       int32_t network_size, int32_t batches_per_mc_run, uint64_t mc_seed, int32_t scheme,
                       int32_t normalization, int32_t dtype, int32_t store_mode, void* paths_dev,
                       int64_t path_pitch, int64_t chunk_contracts, void* targets_dev, void* sync_dev,
                       int64_t sync_bytes, void* stream);
/* Bytes of smc_train_step's sync area for this shape on the current device (128 for whole-contract
 * shapes: a done counter, the status word and the contract queue: the resident kernel's dynamically
 * handed-out last quarter of the rounds, rows_kernel's contracts after each workgroup's first; -1 if
 * the device query fails). */
int64_t smc_train_step_sync_bytes(int32_t timesteps, int32_t network_size, int32_t batches_per_mc_run,
                                  int32_t dtype, int64_t path_pitch);
/* Name of the kernel smc_train_step launches for this shape ("resident_kernel",
 * "resident_kernel(sliced)", or smc_train_targets_kernel's name).  Static string.  dtype may carry
 * SMC_QUERY_RAW: the shape's targets use RAW normalisation (one-wave-per-contract shapes); a bit of its
 * own (ABI 12: it was 0x100, SMC_MATH_HW's bit in smc_normals' dtype); and SMC_MATH_REF (ABI 13). */
#define SMC_QUERY_RAW 0x1000
const char* smc_train_step_kernel(int32_t timesteps, int32_t network_size, int32_t batches_per_mc_run,
                                  int32_t dtype, int64_t path_pitch);
/* Workspace bytes smc_train_targets needs for sliced contracts (0: P too small to slice). */
int64_t smc_engine_workspace_bytes(int64_t chunk_contracts, int32_t timesteps, int64_t n_paths,
                                   int32_t all_rows);
/* Name of the kernel smc_train_targets launches for this shape ("wave_kernel", "resident_kernel",
 * "packed_kernel", the split pairs, "contract_kernel", "queue_kernel" or "rows_ref_kernel+cf_kernel";
 * sliced = a workspace is passed; dtype | SMC_QUERY_RAW | SMC_MATH_REF as for smc_train_step_kernel;
 * "unsupported" for an SMC_MATH_REF shape the engine rejects: f64, a pitch without room for the terminal
 * sum, sliced).  Static string. */
const char* smc_train_targets_kernel(int32_t timesteps, int32_t network_size, int64_t n_paths,
                                     int32_t dtype, int64_t path_pitch, int32_t sliced);
/* Recommended row pitch (elements) for a path scratch buffer of n_paths columns: the row
 * stride becomes an odd multiple of 4 KiB (power-of-two strides alias in HBM). */
int64_t smc_path_pitch(int64_t n_paths, int32_t dtype);
/* The [rows][cols] N(0,1) matrix of contract ordinal m (the values smc_gbm_simulate
 * draws for path p, step t, laid out [t][p]; rows = the contract's T: at T <= 2 one
 * Philox-seeded stream serves 4 consecutive 4-path groups, the stream span of smc_rng.h). */
int32_t smc_normals(uint64_t mc_seed, int64_t ordinal, int32_t rows, int64_t cols,
                    int32_t dtype, void* out_dev, void* stream);

/* ---- correlated multi-asset (basket) engine ---------------------------------
 * Extension of the reference engine (BASELINE.json configs[4]; per-asset dynamics as
 * SimulateBlackScholes, src/spectralmc/gbm.py:224-257, log-Euler; normalisation gbm.py:428-440;
 * targets as _simulate_fft, gbm_trainer.py:806-817) with an equal-weight basket put.
 * contracts_dev: [B][3A+4] f64 rows (K, T, r, rho, X0[A], d[A], v[A]); the equicorrelation
 * matrix (1-rho) I + rho 11^T is Cholesky-factored in LDS per contract.
 * paths_dev: [chunk][A][T][pitch] f32 (SMC_STORE_ALL) or [chunk][A][pitch] (SMC_STORE_TERMINAL),
 * reused per launch of chunk_contracts; terminal_sum_dev (may be NULL): [B][A] f64 sums of the
 * terminal rows; targets_dev: [B][N] complex64.  math: 0 (portable, CPU-reproducible) or
 * SMC_MATH_HW.  Needs 1 <= A <= 8, N % 4 == 0, N <= 4096, N*M a multiple of 2048.
 * sync_dev (may be NULL): smc_basket_sync_bytes(...) bytes, zero-filled before the first call (every
 * call leaves its counters zeroed).  With it, shapes the resident kernel takes (T = 16, N | 4096, N <= 2048,
 * N*M a multiple of 4096 up to 32 x 4096) run basket_resident_kernel per chunk, in which W = N*M /
 * 4096 co-resident workgroups per contract keep the terminal rows on chip and exchange their
 * terminal sums, then basket_mean_fft_kernel over the slices' column sums (reduction orders:
 * oracle_basket_kernel(wg = 1024, slices = W)).  Otherwise, with
 * terminal_sum_dev each chunk is two launches (simulate + store + terminal sums, then the CF pass
 * over the stored terminal rows), without it one fused launch; these two are bit-identical. */
int32_t smc_basket_train_targets(const double* contracts_dev, int64_t n_contracts, int32_t n_assets,
                                 int32_t timesteps, int32_t network_size, int32_t batches_per_mc_run,
                                 uint64_t mc_seed, const int64_t* ordinal_dev, int64_t ordinal0,
                                 int32_t math, int32_t normalization, int32_t store_mode,
                                 void* paths_dev, int64_t path_pitch, int64_t chunk_contracts,
                                 double* terminal_sum_dev, void* targets_dev, void* sync_dev,
                                 int64_t sync_bytes, void* stream);
/* Bytes of smc_basket_train_targets' sync area for this shape and chunk_contracts on the current
 * device (slice-sum exchange + the column sums of one launch; 0: the resident kernel does not take
 * the shape, pass NULL; -1 on a bad argument or a failed query). */
int64_t smc_basket_sync_bytes(int32_t n_assets, int32_t timesteps, int32_t network_size,
                              int32_t batches_per_mc_run, int64_t chunk_contracts);
/* Name of the kernel(s) smc_basket_train_targets launches for this shape ("basket_resident_kernel",
 * "basket_kernel+basket_cf_kernel" or "basket_kernel"); with_sync / keep_sums: whether the call
 * passes sync_dev / terminal_sum_dev.  Static string. */
const char* smc_basket_train_targets_kernel(int32_t n_assets, int32_t timesteps, int32_t network_size,
                                            int32_t batches_per_mc_run, int32_t with_sync, int32_t keep_sums);
/* Basket workgroups (one per contract) resident on the current device at once, for sizing
 * chunk_contracts in whole rounds; -1 on a bad argument or a failed device query. */
int64_t smc_basket_resident_slots(int32_t n_assets, int32_t network_size, int32_t math);

/* ---- complex-valued MLP training step --------------------------------------
 * Replaces the network half of _torch_step (src/spectralmc/gbm_trainer.py:819-835) for
 * ComplexSequential chains of ComplexLinear (cvnn.py:65-143) with optional modReLU
 * (cvnn.py:168-210) or zReLU (cvnn.py:149-162) activations.  Parameters, gradients and Adam
 * moments are flat buffers in the model's parameter order; a layer names its tensors by
 * element offset into them (-1 = absent). */
#define SMC_CVNN_MAX_LAYERS 8
#define SMC_ACT_NONE     0
#define SMC_ACT_MODRELU  1
#define SMC_ACT_ZRELU    2

typedef struct smc_cvnn_layer {
  int32_t in_features, out_features;
  int32_t activation;            /* SMC_ACT_* applied after this layer's affine map */
  int32_t reserved;
  int64_t w_re, w_im;            /* [out][in] real_weight / imag_weight offsets        */
  int64_t b_re, b_im;            /* [out] real_bias / imag_bias offsets or -1          */
  int64_t act_bias;              /* [out] modReLU bias offset or -1                    */
} smc_cvnn_layer;

/* Where an Adam update also writes the matrix-core (MFMA) operand copies of the weights it changes, so the
 * next smc_cvnn_mfma_forward_backward skips its pack launch (mode | SMC_CVNN_MFMA_PACKED): each complex
 * weight w = a + i b of layer l lands at Wc[2j][2k] = Wc[2j+1][2k+1] = a, Wc[2j][2k+1] = -b, Wc[2j+1][2k] = b
 * and at the same places of Wc^T (smc_cvnn_mfma_pack_plan fills it from the forward_backward plan). */
typedef struct smc_cvnn_pack_layer {
  int64_t w_re, w_im;            /* the layer's weight offsets in params (as smc_cvnn_layer)   */
  int32_t ni, no;                /* complex in / out features                                  */
  int32_t win, wout;             /* packed widths (2 ni, 2 no rounded up to the K block)       */
  int64_t wc, wct;               /* element offsets of Wc [wout][win] and Wc^T [win][wout]     */
} smc_cvnn_pack_layer;
typedef struct smc_cvnn_pack {
  void* ws;                      /* the forward_backward workspace                             */
  int32_t bf16;                  /* operands are bf16 (SMC_CVNN_MFMA_BF16), else f32           */
  int32_t n_layers;              /* 0: nothing to write                                        */
  smc_cvnn_pack_layer layer[SMC_CVNN_MAX_LAYERS];
} smc_cvnn_pack;

/* torch.optim.Adam (defaults of gbm_trainer.py:1513) on flat buffers; `step` is torch's
 * capturable f32 step counter, read before and incremented after the update. */
typedef struct smc_adam_args {
  void* params;
  void* exp_avg;
  void* exp_avg_sq;
  float* step;
  double lr, beta1, beta2, eps, weight_decay;
  double* norm_partials;         /* [smc_adam_norm_partials(n_params)] scratch, ZEROED before
                                    the first call (its last slot is the fused finalize's
                                    arrival counter; every COMPLETED call leaves it zero:
                                    a caller that allocates it without zeroing, or reuses
                                    it after a launch that did not complete, must zero it
                                    again, else no workgroup counts as last and grad_norm,
                                    loss and step stop being written)                      */
  void* grad_norm;               /* scalar out: ||grad||_2 (gbm_trainer.py:834)         */
  void* loss;                    /* scalar out: grads[n_params] (the loss slot)         */
  const smc_cvnn_pack* pack;     /* or NULL: the update also writes these packed copies (ABI 13) */
} smc_adam_args;

/* Number of per-workgroup gradient partials ([blocks][n_params + 1]) for this batch. */
int32_t smc_cvnn_plan(const smc_cvnn_layer* layers, int32_t n_layers, int32_t dtype, int64_t batch,
                      int64_t* partial_blocks);
/* Forward, loss = mse(Re) + mse(Im), backward: partials[g] = the gradients and loss share
 * of workgroup g's rows.  input_im may be NULL (zeros); targets [batch][N] complex. */
int32_t smc_cvnn_forward_backward(const smc_cvnn_layer* layers, int32_t n_layers, int32_t dtype,
                                  const void* params, int64_t n_params, const void* input_re,
                                  const void* input_im, const void* targets, int64_t batch,
                                  void* partials, int64_t partial_blocks, void* stream);
/* grads[0..n_params] = fixed-order sum of the partials (last entry: loss).  With adam != NULL
 * the Adam update, grad norm, loss copy and step increment follow (ABI 12: for networks of up to
 * 65,535 parameters in the same launch, whose last workgroup takes the grad norm, loss and step;
 * larger ones in a second, one-workgroup launch). */
int32_t smc_cvnn_reduce_grads(int32_t dtype, const void* partials, int64_t partial_blocks,
                              int64_t n_params, void* grads, const smc_adam_args* adam, void* stream);
/* Adam update from an already reduced (e.g. all-reduced) grads[0..n_params]. */
int32_t smc_adam_step(int32_t dtype, int64_t n_params, const void* grads, const smc_adam_args* adam,
                      void* stream);
/* f64 entries of smc_adam_args.norm_partials: one per 64 gradient entries + the arrival counter. */
int64_t smc_adam_norm_partials(int64_t n_params);

/* ---- the same network step on the matrix cores (csrc/cvnn_mfma.hip) ---------
 * Each complex layer runs as real GEMMs of the interleaved (re, im) vectors on MFMA:
 *   SMC_CVNN_MFMA_F32   f32 operands (v_mfma_f32_16x16x4_f32), the network's own precision;
 *   SMC_CVNN_MFMA_BF16  bf16 operands rounded to nearest even, f32 accumulation, f32 master
 *                       parameters / activations / loss / Adam (BASELINE configs[2] "bf16 CVNN";
 *                       an extension: the reference asserts full precision, gbm_trainer.py:679-686).
 * Parameters, inputs and targets are f32 / complex64.  The call writes per-segment partials
 * [partial_blocks][n_params + 1] (gradients, loss last) that smc_cvnn_reduce_grads(SMC_DTYPE_F32,
 * ...) sums in order, exactly as after smc_cvnn_forward_backward.  Shapes whose widths exceed the
 * kernels' LDS plan return SMC_ERR_INVALID_SHAPE from the plan (callers keep the VALU kernels). */
#define SMC_CVNN_MFMA_F32   1
#define SMC_CVNN_MFMA_BF16  2
#define SMC_CVNN_MFMA_PACKED 0x100  /* flag, OR into forward_backward's mode: the workspace already holds
                                       the packed weights of params (the last Adam update wrote them).
                                       Valid only while params change through those updates alone: a
                                       caller that writes params any other way (a state_dict load, a
                                       broadcast) must drop the flag for the next call (net.py
                                       FusedNetworkStep.invalidate_pack) */
int32_t smc_cvnn_mfma_plan(const smc_cvnn_layer* layers, int32_t n_layers, int32_t mode, int64_t batch,
                           int64_t* partial_blocks, int64_t* workspace_bytes);
int32_t smc_cvnn_mfma_forward_backward(const smc_cvnn_layer* layers, int32_t n_layers, int32_t mode,
                                       const float* params, int64_t n_params, const float* input_re,
                                       const float* input_im, const void* targets, int64_t batch,
                                       float* partials, int64_t partial_blocks, void* workspace,
                                       int64_t workspace_bytes, void* stream);
/* The packed-weight layout of that plan for Adam (smc_adam_args.pack); out->n_layers = 0 for plans whose
 * wide layers keep their own pack launch (the layered GEMM path). */
int32_t smc_cvnn_mfma_pack_plan(const smc_cvnn_layer* layers, int32_t n_layers, int32_t mode, int64_t batch,
                                void* workspace, smc_cvnn_pack* out);

#ifdef __cplusplus
}
#endif

#endif /* SPECTRALMC_HIP_H */
