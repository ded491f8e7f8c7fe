/*
 * wavernn_mi355x.h -- C-ABI of the MI355X-native WaveRNN vocoder (libwavernn_mi355x.so).
 *
 * Drop-in boundary for the reference's vocoder inference path. Each entry point names the
 * reference interface it replaces (paths relative to RuntimeRacer/Real-Time-Voice-Cloning):
 *
 *   reference                                                   this ABI
 *   -----------------------------------------------------------  -------------------------------
 *   WaveRNNVocoder.Vocoder()        libwavernn/<variant>/src/     wrnn_create
 *                                   WaveRNNVocoder.cpp:17-21
 *   Vocoder.loadWeights(path)       WaveRNNVocoder.cpp:22-31       wrnn_load_bin (.bin image), or
 *                                                                   wrnn_load_tensor + wrnn_finalize
 *   model.load_state_dict(sd)       vocoder/inference.py:35        (state-dict names, PyTorch layout)
 *   Vocoder.setRandomSeed(seed)     WaveRNNVocoder.cpp:33-35       wrnn_set_seed
 *   torch.manual_seed(seed)         vocoder/inference.py:97-101
 *   Vocoder.melToWav(mels)          WaveRNNVocoder.cpp:37-47       wrnn_generate (host buffers)
 *   WaveRNN.generate(mels, batched, vocoder/models/                 wrnn_generate / _device
 *     target, overlap, ...)         fatchord_version.py:155-240    (device loop; the f64 cross-fade,
 *                                   runtimeracer_version.py:199-295 mu-law and de-emphasis stay on
 *                                                                   the host, :242-255)
 *   fold_with_overlap arithmetic    fatchord_version.py:316-327    wrnn_fold_shape
 *   RuntimeError("Model hasn't been loaded ...")  WaveRNNVocoder.cpp:39-41   WRNN_ERR_NOT_LOADED +
 *   RuntimeError("Cannot open file.")             WaveRNNVocoder.cpp:24-26   wrnn_last_error()
 *
 * Conventions: plain C types only; every function returns 0 on success and a negative
 * WRNN_ERR_* code on failure, with a thread-local message from wrnn_last_error(). Nothing
 * throws or aborts across the ABI. A handle owns its device memory and HIP stream and must be
 * used by one thread at a time; distinct handles are independent (one per GPU / per caller
 * thread), unlike the reference's shared static RNG (net_impl.cpp:136).
 *
 * Sampling noise follows the Philox4x32-10 contract documented in DESIGN.md ("RNG contract"):
 * identical (seed, stream) -> identical outputs on any device.
 */
#ifndef WAVERNN_MI355X_H
#define WAVERNN_MI355X_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define WRNN_OK 0
#define WRNN_ERR_INVALID (-1)    /* bad argument / unsupported hyper-parameters        */
#define WRNN_ERR_NOT_LOADED (-2) /* generate before finalize (WaveRNNVocoder.cpp:39-41) */
#define WRNN_ERR_HIP (-3)        /* HIP runtime error                                   */
#define WRNN_ERR_OOM (-4)        /* device allocation failed                            */
#define WRNN_ERR_ABORTED (-5)    /* progress callback returned non-zero                 */
#define WRNN_ERR_CAPACITY (-6)   /* caller's output buffer too small                    */

#define WRNN_MODEL_FATCHORD 0     /* 'fatchord-wavernn'     vocoder/models/base.py:13 */
#define WRNN_MODEL_RUNTIMERACER 1 /* 'runtimeracer-wavernn' vocoder/models/base.py:15 */
#define WRNN_MODEL_GENEING 2      /* 'geneing-wavernn'      vocoder/models/base.py:14 */

#define WRNN_MODE_RAW 0 /* softmax over 2**bits classes, Categorical sample (geneing: 'BITS') */
#define WRNN_MODE_MOL 1 /* 10-component discretized mixture of logistics   */
#define WRNN_MODE_BETA 2 /* geneing 'RAW': Beta(exp(l0), exp(l1)) on 2 outputs
                            (geneing_version.py:95-96,207-210, distribution.py:7-20) */

/* Recurrence engines (same results, different schedules):
 *   CHAIN   one launch per layer group per step, HIP-graph captured (every topology)
 *   PERSIST one persistent weight-stationary launch per row batch, 8 XCD-local groups
 *           (fatchord 512 / runtimeracer 256 dims, n_classes <= 1024, any row count)
 *   AUTO    PERSIST when the call qualifies, else CHAIN (default; env WRNN_ENGINE overrides) */
#define WRNN_ENGINE_AUTO 0
#define WRNN_ENGINE_CHAIN 1
#define WRNN_ENGINE_PERSIST 2

/* Topology, with the field names of config/hparams.py:220-285 / :356-421. */
typedef struct wrnn_config {
    int model_type;         /* WRNN_MODEL_*                         */
    int mode;               /* WRNN_MODE_*                          */
    int bits;               /* RAW: n_classes = 2**bits             */
    int rnn_dims;           /* 512 fatchord, 256 runtimeracer       */
    int fc_dims;
    int compute_dims;       /* MelResNet width (128)                */
    int res_out_dims;       /* aux width (128); aux_dims = /4       */
    int res_blocks;         /* 10                                   */
    int pad;                /* 2                                    */
    int feat_dims;          /* num_mels (80)                        */
    int hop_length;         /* 200 = prod(upsample_factors)         */
    int n_upsample;         /* number of upsample stages (3)        */
    int upsample_factors[4];/* (5, 5, 8)                            */
} wrnn_config;

typedef struct wrnn_handle wrnn_handle;

/* Called at i = 0, 100, 200, ... < seq_len, in order, once each, with the reference's
 * progress_callback arguments (fatchord_version.py:234-236): step index i, seq_len, b_size,
 * gen_rate in kHz -- as soon as every fold row has finished step i (PERSIST: the kernels
 * publish their step count to host-mapped memory; CHAIN: between 100-step graphs). Return
 * non-zero to abort (WRNN_ERR_ABORTED): no further callbacks; PERSIST sets a host-mapped abort
 * word that every XCD group checks at its next progress point, so the launches drain within
 * ~100 steps (the reference stops at the raising step). */
typedef int (*wrnn_progress_fn)(void* user, int i, int seq_len, int b_size, double gen_rate_khz);

/* Library / device info. */
const char* wrnn_version(void);
const char* wrnn_last_error(void);
int wrnn_device_count(int* count);

/* Create a vocoder bound to HIP device `device`. */
int wrnn_create(const wrnn_config* cfg, int device, wrnn_handle** out);
void wrnn_destroy(wrnn_handle* h);

/* Load one state-dict tensor (fp32, PyTorch layout/shape, host memory); names as in the
 * reference state_dict, e.g. "rnn1.weight_ih_l0", "upsample.resnet.conv_in.weight".
 * Unknown names (e.g. "step") are ignored; shape mismatches are WRNN_ERR_INVALID. */
int wrnn_load_tensor(wrnn_handle* h, const char* name, const float* data, const int64_t* shape,
                     int ndim);
/* Check every required tensor is present and repack them into the device layout. */
int wrnn_finalize(wrnn_handle* h);

/* libwavernn ".bin" weight files -- the second on-disk format of the reference, written by
 * vocoder/libwavernn/convert.py:14-58 (dense or Pruner 1x4 block-compressed matrices) and read
 * by Vocoder.loadWeights (WaveRNNVocoder.cpp:22-31, wavernn.cpp:37-184).
 * wrnn_bin_read parses a whole file image (host memory) for the topology in `cfg` and hands
 * every tensor to `fn` under its state-dict name, densified, in PyTorch layout; host only, no
 * device is touched. A non-zero return of `fn` stops the read and is returned.
 * wrnn_load_bin = wrnn_bin_read into wrnn_load_tensor, then wrnn_finalize. Format or shape
 * mismatches are WRNN_ERR_INVALID ("libwavernn .bin: ..."). */
typedef int (*wrnn_tensor_fn)(void* user, const char* name, const float* data,
                              const int64_t* shape, int ndim);
int wrnn_bin_read(const void* data, size_t bytes, const wrnn_config* cfg, wrnn_tensor_fn fn,
                  void* user);
int wrnn_load_bin(wrnn_handle* h, const void* data, size_t bytes);

/* Seed of the Philox noise; resets the per-call stream counter (torch.manual_seed). */
int wrnn_set_seed(wrnn_handle* h, uint64_t seed);
/* Explicit stream id for the next call (advanced by one per utterance afterwards). */
int wrnn_set_stream(wrnn_handle* h, uint32_t stream);
/* Stream id the next call's first utterance will use. */
int wrnn_get_stream(wrnn_handle* h, uint32_t* stream);
/* Explicit noise stream of each utterance of the NEXT generate call only (n = its n_utts;
 * n = 0 clears): utterance u draws from stream streams[u] instead of (stream + u), and the
 * counter moves past the largest one afterwards. This is what makes sharded inference
 * world-size invariant: every rank gives utterance i of the global batch the stream
 * (base + i), as the reference's CPU backend seeds every worker instance explicitly
 * (vocoder/libwavernn/inference.py:106-108, :200-204). A count that does not match the
 * call's n_utts makes that call fail with WRNN_ERR_INVALID. */
int wrnn_set_utt_streams(wrnn_handle* h, const uint32_t* streams, int n);
/* Fold range of each utterance of the NEXT wrnn_generate_batch_device call only (n = its
 * n_utts; n = 0 clears): utterance u runs only its fold rows lo[u] .. hi[u] - 1 (0 <= lo < hi
 * <= num_folds, batched calls), as rows row_offset[u] .. row_offset[u + 1] - 1 of the output.
 * Each row computes exactly what it computes in a full call -- same conditioning positions
 * (fold_with_overlap, fatchord_version.py:290-340), same noise words (Philox keyed by the
 * global fold index) -- so the fold rows of one utterance can be split over ranks and the
 * union equals the single-call rows bit for bit (the "one exchange step" single-utterance
 * split of SURVEY §8e). The reference has no such call: its folds always run as one batch
 * (fatchord_version.py:180-187). wrnn_generate refuses an armed range. */
int wrnn_set_fold_ranges(wrnn_handle* h, const int* lo, const int* hi, int n);

/* Fold arithmetic of fold_with_overlap for a mel of n_frames frames
 * (upsampled length L = n_frames * hop). batched=0 -> one row of L steps. */
int wrnn_fold_shape(int n_frames, int hop_length, int batched, int target, int overlap,
                    int* num_folds, int* seq_len);

/* Generate one utterance. mel: host float32 (feat_dims, n_frames) row-major, ALREADY
 * normalised (divided by max_abs_value, vocoder/inference.py:91-92).
 * Outputs per fold row, row-major (num_folds, seq_len):
 *   RAW: labels[b*seq_len+i] (int16 class index) and/or samples (float32 2k/(n-1)-1)
 *   MOL: samples (float32 in [-1, 1]); labels must be NULL.
 * `capacity` = elements available in each non-NULL output buffer. */
int wrnn_generate(wrnn_handle* h, const float* mel, int n_frames, int batched, int target,
                  int overlap, int16_t* labels, float* samples, size_t capacity,
                  int* num_folds, int* seq_len, wrnn_progress_fn cb, void* user);

/* Batched multi-utterance generation with inputs resident in HBM: mels[u] are DEVICE
 * pointers to (feat_dims, n_frames[u]) float32. Rows of all utterances run as one batch of
 * sum(num_folds) rows; row_offset[u] (host, n_utts+1 entries, filled by the call) gives each
 * utterance's first row. Outputs are DEVICE buffers of (total_rows, seq_len). Utterance u
 * uses noise stream (stream + u), or streams[u] after wrnn_set_utt_streams. Results are
 * identical to n_utts single calls with those streams. */
int wrnn_generate_batch_device(wrnn_handle* h, int n_utts, const float* const* mels,
                               const int* n_frames, int batched, int target, int overlap,
                               int16_t* labels_dev, float* samples_dev, size_t capacity,
                               int* row_offset, int* seq_len, wrnn_progress_fn cb, void* user);

/* Select the recurrence engine for later calls (WRNN_ENGINE_*). Requesting PERSIST for a
 * call that does not qualify makes that call fail with WRNN_ERR_INVALID. */
int wrnn_set_engine(wrnn_handle* h, int engine);
/* Engine that ran the last call. */
int wrnn_last_engine(wrnn_handle* h, int* engine);
/* Calls on this handle that fell back from PERSIST to CHAIN under WRNN_ENGINE_AUTO (the
 * persistent launch could not run, e.g. its 256 workgroups did not become co-resident), and
 * the last reason (NUL-terminated, truncated to reason_cap). Each fallback also prints a
 * warning to stderr; with WRNN_ENGINE_PERSIST requested the call fails instead. AUTO stops
 * trying PERSIST after 3 failed calls in a row. */
int wrnn_fallback_info(wrnn_handle* h, int* count, char* reason, size_t reason_cap);
/* Block-sparse execution of pruned checkpoints (the reference's Pruner, vocoder/pruner.py:60-88;
 * its native backend's sparse GEMV, vocoder/libwavernn/runtimeracer_version/src/wavernn.cpp:
 * 162-184): *available = the loaded fatchord weights have a sparse k_persist image (their live
 * 1 x 4 blocks fit the kernel's LDS lists); *last_call = the last call's register-resident
 * launches ran it; *density = live fraction of the step matrices' 1 x 4 blocks; *fill_f4 = the
 * fullest slot's list size (float4). Results equal the dense kernels' bit for bit. Env
 * WRNN_SPARSE=0 turns it off. Any pointer may be null. */
int wrnn_sparse_info(wrnn_handle* h, int* available, int* last_call, double* density, int* fill_f4);
/* Launch-planner rates (operator tuning; no reference equivalent): the per-step
 * costs the planner minimises, as text lines `key v1 v2 ...` ('#' comments; keys and meaning in
 * DESIGN.md). A handle starts from the built-in measured defaults overridden by env WRNN_RATES
 * (a file) or rates_mi355x.txt beside the library. wrnn_set_rates overrides keys of the
 * defaults (NULL: reload as at creation; a bad table is WRNN_ERR_INVALID and changes nothing);
 * wrnn_get_rates writes the table in effect, with its source, NUL-terminated. */
int wrnn_set_rates(wrnn_handle* h, const char* table);
int wrnn_get_rates(wrnn_handle* h, char* buf, size_t cap);
/* Host-only launch plan (no device): the plan wrnn_generate would make for `rows` fold rows of
 * `seq_len` steps of a model_type / bits / mode model under the rate table `table` (NULL: the
 * built-in defaults), every kernel variant taken as spill-free. flags: 1 sparse image, 2 P1 ring /
 * per-frame P1, 4 wide images, 8 sparse forced (WRNN_SPARSE=1). Outputs: launches, rows per group and wide flag of the first `cap`,
 * and the row rotation's launch count (0: none). */
int wrnn_debug_plan(const char* table, int model_type, int bits, int mode, int rows, int seq_len, int flags,
                    int* n_launches, int* rows_per_group, int* wide, int cap, int* rot_launches);
/* Launch plan of the last PERSIST call (operator introspection; no reference equivalent):
 * *n_launches launches; for i < n_launches, launch i runs fold rows first_row[i] + g + 8 r,
 * r < rows_per_group[i], on the wide MFMA kernel when wide[i] != 0. Arrays may be null;
 * at most `cap` entries are written. 0 launches after a CHAIN call. */
int wrnn_plan_info(wrnn_handle* h, int* n_launches, int* first_row, int* rows_per_group, int* wide,
                   int cap);

/* Per-stage timing of the dominant recurrent kernel. Enable before a call; read after:
 * average duration in microseconds of the launches of stage `stage` in the last call, and
 * the number of launches averaged. CHAIN: in-kernel s_memrealtime stamps (100 MHz) of every
 * 8th step. PERSIST: one stage, HIP events recorded on the launch stream around each launch. */
int wrnn_enable_stage_timing(wrnn_handle* h, int enable);
int wrnn_stage_timing(wrnn_handle* h, int stage, double* avg_us, int* launches);
/* Name and algorithmic bytes / FLOPs per launch of stage `stage` for the last call's shape. */
int wrnn_stage_info(wrnn_handle* h, int stage, char* name, size_t name_cap, double* bytes,
                    double* flops, int* n_stages);

/* Host post-processing helper (no device): de_emphasis of the reference,
 * scipy.signal.lfilter([1], [1, -coef], x) (vocoder/audio.py:92-93, applied in
 * fatchord_version.py:251-252), same doubles bit for bit. y may alias x. */
int wrnn_de_emphasis(const double* x, double* y, size_t n, double coef);

/* Host post-processing of categorical fold rows (no device), fatchord_version.py:238-255 with
 * labels (nf, S) int16 from a batched RAW generate: xfade_and_unfold
 * (fatchord_version.py:342-404), decode_mu_law (vocoder/audio.py), de_emphasis and the final
 * fade, same doubles bit for bit as the reference's numpy / scipy path.
 * wrnn_post_overlaps: the nf + 1 cross-faded overlap regions ((nf + 1) * overlap doubles), from
 * samp[k] = the f64 value of label k (2k/(n-1) - 1 in fp32) and the fade_in / fade_out vectors
 * of xfade_and_unfold; the caller decodes them (mu-law) itself.
 * wrnn_post_assemble: the first n_out unfolded samples from mid_lut[k] (the value of a fold
 * middle sample with label k) and the decoded regions, then de_emphasis (if preemph) and
 * out[n_out - fade_len + i] *= fade[i]. Labels outside [0, n_classes) -> WRNN_ERR_INVALID. */
int wrnn_post_overlaps(const int16_t* labels, int nf, int S, int overlap, const double* samp,
                       int n_classes, const double* fade_in, const double* fade_out,
                       double* regions);
int wrnn_post_assemble(const int16_t* labels, int nf, int S, int overlap, const double* mid_lut,
                       int n_classes, const double* regions, int preemph, double coef,
                       const double* fade, size_t fade_len, double* out, size_t n_out);

/* Host restatement of the BETA noise contract (no device): the sample of one (step, row)
 * for Beta(alpha, beta), rescaled to [-1, 1] -- the value the kernels compute (tests). */
int wrnn_debug_beta(uint64_t seed, uint32_t stream, uint32_t step, uint32_t row, float alpha,
                    float beta, float* out);

/* Host restatement of the RAW decision every kernel makes (csrc/cand_key.h): for
 * the n_classes logits of one (step, fold, stream) row, the class argmax_k (l_k + G_k), G_k =
 * -log q_k of the Philox contract's Exp(1) variate (philox.h gumbel_q_of: float64 logs, fixed
 * point to 2^-27), l + G formed exactly -- the reference's argmax((softmax(l)/sum)/q) without
 * fp32 rounding of its own. `margin` (may be NULL) receives the float64 value of the decision's
 * top-1 minus top-2 l + G (how far it was from a flip). No device needed (tests). */
int wrnn_debug_decide(uint64_t seed, uint32_t stream, uint32_t step, uint32_t fold, const float* logits,
                      int n_classes, int* label, double* margin);

/* Row rotation of the persistent engine: the plan for R fold rows of S steps
 * given the per-step costs of groups of q + 1 and q rows (q = R / 8), without a device. On
 * success *launches = K > 0, *n_hi / *n_lo = the steps a group of q + 1 / q rows runs per
 * launch, and vmap (capacity K * 8 * (q + 1) pairs, may be NULL) receives per launch and
 * virtual row v = g + 8 r the (physical row, step offset) pair, (-1, -1) for the row slots a
 * q-row group leaves empty; *launches = 0 when no rotation pays (tests). */
int wrnn_debug_rot_plan(int rows, int seq_len, double us_hi, double us_lo, int* launches, int* n_hi,
                        int* n_lo, int* vmap, size_t capacity);
/* Time-sliced wide launches for R fold rows of S steps, without a device: on
 * success *launches = K > 0 (0 = the plan does not apply), per launch k rows_steps[2 k] = rows per
 * group and rows_steps[2 k + 1] = steps (capacity >= 2 K), and vmap (capacity >= K * 8 * 16
 * pairs, may be NULL) the (physical row, step offset) of virtual row v = g + 8 r at
 * [(k * 128 + v) * 2], (-1, -1) beyond the launch's rows (tests). */
int wrnn_debug_slice_plan(int rows, int seq_len, int* launches, int* rows_steps, size_t rs_capacity, int* vmap,
                          size_t capacity);
/* The rotation of the last persistent call: launches (0 = none), steps per launch of the q + 1 /
 * q-row groups. */
int wrnn_rot_info(wrnn_handle* h, int* launches, int* n_hi, int* n_lo);
/* Steps per launch, averaged over the launches of stage `stage` (wrnn_stage_info's index) of the
 * last persistent call: the call's S for row batches, less for rotated / time-sliced launches
 * (DESIGN.md §3.0e-f). */
int wrnn_persist_steps(wrnn_handle* h, int stage, double* steps_per_launch);

/* Host-side exhaustive check of the wide launch's exchange layout (kernels_persist_wide.hip,
 * csrc/wide_layout.h) for a group of `rows_per_group` rows (1..16): returns the number of
 * violations (0 = every producer packet of a hop lands on exactly the consumer packet that
 * expects its (row, unit quad), aligned, inside its slot; no-packet offsets out of range),
 * or WRNN_ERR_INVALID. No device needed. */
int wrnn_debug_wide_layout(int rows_per_group);

/* Raw access for tests: copy the RAW noise (seq_len, rows, n_classes) of the last call's
 * first `n_steps` steps to host (float32). */
int wrnn_debug_noise(wrnn_handle* h, int n_steps, float* out, size_t capacity);
/* Copy the upsampled conditioning of the last call to host: mel (L, feat) and aux
 * (n_frames, res_out_dims) per utterance 0. */
int wrnn_debug_upsample(wrnn_handle* h, float* mel_out, size_t mel_cap, float* aux_out,
                        size_t aux_cap);
/* Copy the PERSIST conditioning input P1 of the last persistent call for (step, fold row):
 * 4 * rnn_dims floats, unit-major (r, z, n of W_ih1 (I c) + b_ih1, then I c + b_I) -- the
 * per-frame form (taps of the upsampler over per-frame projections) the engines consume.
 * WRNN_ERR_INVALID when the last call did not run the persistent engine. */
int wrnn_debug_p1(wrnn_handle* h, int step, int row, float* out, size_t capacity);

/* Teacher-forced logit gate (SURVEY §7 "Hard parts" iii): later calls record the
 * pre-sampling logits -- output of the last linear layer plus its bias, what the reference
 * feeds to softmax / the MoL sampler (fatchord_version.py:213, runtimeracer_version.py:270) --
 * of every fold row at up to 8 steps (n = 0 turns recording off). Recorded by the kernels that
 * run the call (every persistent kernel and the CHAIN sampler); off, it costs one uniform
 * branch per step. wrnn_debug_logits copies n_classes floats of (step, fold row) of the last
 * call; WRNN_ERR_INVALID when that step was not recorded. */
int wrnn_set_debug_steps(wrnn_handle* h, const int* steps, int n);
int wrnn_debug_logits(wrnn_handle* h, int step, int row, float* out, size_t capacity);

#ifdef __cplusplus
}
#endif
#endif /* WAVERNN_MI355X_H */
