/*
 * libpcx — MI355X (gfx950) native kernels for the phoneme-contrast train step.
 *
 * C ABI only: plain pointers, sizes and a hipStream_t.  Every entry point is asynchronous on
 * the given stream, never allocates or frees device memory (the caller passes workspaces sized
 * by the matching *_workspace_bytes query), never synchronises the device, and returns
 * PCX_OK or a negative error code; pcx_last_error() gives the message of the last failure on the
 * calling thread.
 *
 * Reference interfaces replaced (paths relative to the reference checkout):
 *   pcx_supcon_*      SupervisedContrastiveLoss.forward + its autograd backward
 *                     (src/training/losses.py:41-86); NTXentLoss labelled branch
 *                     (losses.py:101-151) is the same call with base_temperature = temperature.
 *   pcx_net_*         PhonemeNet.forward (src/models/phoneme_cnn.py:98-126) and
 *                     PhonemeNetDeep.forward (phoneme_cnn.py:274-304) with their autograd
 *                     backward, train (batch-stat BatchNorm, Dropout2d) and eval mode.
 *   pcx_adam_step     torch.optim.Adam.step with coupled weight decay as configured at
 *                     scripts/train.py:129-133.
 */
#ifndef PCX_H_
#define PCX_H_

#include <stddef.h>
#include <stdint.h>

#include <hip/hip_runtime_api.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PCX_OK 0
#define PCX_EINVAL (-1)   /* bad argument / unsupported configuration */
#define PCX_ESHAPE (-2)   /* tensor shape does not match the plan     */
#define PCX_EHIP (-3)     /* HIP runtime error (launch failure, ...)  */
#define PCX_EWORKSPACE (-5) /* workspace smaller than *_workspace_bytes */

#define PCX_REDUCTION_MEAN 0
#define PCX_REDUCTION_SUM 1
#define PCX_REDUCTION_NONE 2

/* library version (major*10000 + minor*100 + patch) */
int pcx_version(void);
/* copies the last error message of this thread into buf (NUL-terminated); returns its length */
int pcx_last_error(char* buf, size_t n);

/* ------------------------------------------------------------------ SupCon / NT-Xent loss
 * features [B,D] fp32 row-major (assumed L2-normalised), labels [B] int64 or NULL,
 * mask [B,B] fp32 row-major or NULL (exactly one of labels/mask must be given).
 * Forward writes loss_out ([1] for mean/sum, [B] for none) and rowstats [B*4] (kept by the
 * caller for the backward).  Backward writes dfeatures [B,D] = d(sum_i w_i loss_i)/dF where
 * w_i comes from grad_out ([1] for mean/sum, [B] for none). */
size_t pcx_supcon_workspace_bytes(int64_t B, int64_t D);
int pcx_supcon_forward(const float* features, const int64_t* labels, const float* mask,
                       int64_t B, int64_t D, float temperature, float base_temperature,
                       int reduction, float* loss_out, float* rowstats,
                       void* workspace, size_t workspace_bytes, hipStream_t stream);
int pcx_supcon_backward(const float* features, const int64_t* labels, const float* mask,
                        int64_t B, int64_t D, float temperature, float base_temperature,
                        int reduction, const float* grad_out, const float* rowstats,
                        float* dfeatures, void* workspace, size_t workspace_bytes,
                        hipStream_t stream);

/* Anchor-row ranges (the global-batch mode): rows [row0, row0+nrows) of a batch of B
 * features act as anchors against all B columns.  A partition of [0, B) over ranks reproduces the
 * single-batch loss: forward_rows writes rowstats [nrows*4] and loss_out ([1]: the range's share
 * of the batch mean or sum; [nrows] for none).  coef_rows turns the range's rowstats + grad_out
 * ([1] or [nrows]) into coef [nrows*4]; backward_rows takes coef for ALL B rows (the ranges'
 * coefficients gathered) and writes dfeatures [nrows,D] = the full d loss / dF of its rows (the
 * anchor-side and column-side terms both: no reduction of dF across ranges is needed).  The
 * single-range calls above are row0 = 0, nrows = B.  Replaces nothing in the reference (which is
 * single-device, src/training/losses.py:41-86); the semantics are that of the reference loss on
 * the concatenated batch. */
size_t pcx_supcon_rows_workspace_bytes(int64_t B, int64_t D, int64_t nrows);
int pcx_supcon_forward_rows(const float* features, const int64_t* labels, const float* mask,
                            int64_t B, int64_t D, int64_t row0, int64_t nrows, float temperature,
                            float base_temperature, int reduction, float* loss_out, float* rowstats,
                            void* workspace, size_t workspace_bytes, hipStream_t stream);
int pcx_supcon_coef_rows(const float* rowstats, const float* grad_out, int64_t B, int64_t nrows,
                         float base_temperature, int reduction, float* coef, hipStream_t stream);
int pcx_supcon_backward_rows(const float* features, const int64_t* labels, const float* mask,
                             int64_t B, int64_t D, int64_t row0, int64_t nrows, float temperature,
                             float base_temperature, const float* coef, float* dfeatures,
                             void* workspace, size_t workspace_bytes, hipStream_t stream);

/* ------------------------------------------------------------------ Adam (flat buffers)
 * p, g, m, v: n fp32 each.  Coupled L2 (g += wd*p), bias correction with 1-based `step`.
 * grad_scale multiplies g first (1/world_size after an all-reduce SUM). */
int pcx_adam_step(float* p, const float* g, float* m, float* v, int64_t n, int64_t step,
                  float lr, float beta1, float beta2, float eps, float weight_decay,
                  float grad_scale, hipStream_t stream);


/* ------------------------------------------------------------------ whole-network plans
 * A plan fixes the network configuration and the input shape [B, 1, F, T]; it owns no device
 * memory.  Parameters are passed as an array of device pointers in the reference's
 * model.named_parameters() order, gradients in the same order; bn_stats holds
 * {running_mean, running_var} of every BatchNorm in state_dict order (2 pointers per BN) and
 * bn_counts their num_batches_tracked (int64).  dropout[i] is a [B][C_i] keep-scale mask
 * (0 or 1/(1-p)) per nn.Dropout2d in forward order, or NULL (no dropout).  The forward leaves
 * the activations the backward needs inside `workspace`, so forward and backward of one step
 * must share it. */
#define PCX_NET_CNN_SMALL 0  /* "phoneme_cnn"      PhonemeNet     */
#define PCX_NET_CNN_DEEP 1   /* "phoneme_cnn_deep" PhonemeNetDeep */

typedef struct pcx_net_config {
    int kind;
    int in_channels;      /* must be 1 */
    int embedding_dim;
    int use_attention;
    int hidden_dims[4];   /* deep only */
    int use_residual;     /* deep only */
    int conv_bf16;        /* deep only: conv operands rounded to bf16, float32 accumulation (0: fp32) */
} pcx_net_config;

/* The cnn_deep convolution engine as a standalone op (src/models/phoneme_cnn.py:146-304 convs):
 * mode 0  out = conv2d(x, w)                      x [B][cin][IH][IW], w [cout][cin][k][k], out [B][cout][OH][OW]
 * mode 1  out (+)= d conv2d / d x  applied to dy  dy [B][cout][OH][OW], out [B][cin][IH][IW] (+= if accumulate)
 * mode 2  out = d conv2d / d w  applied to dy     out [cout][cin][k][k]; ws >= pcx_conv2d_workspace_bytes
 * precision 0: float32 operands; 1: operands rounded to bf16, float32 accumulation.  Deterministic. */
size_t pcx_conv2d_workspace_bytes(int mode, int precision, int B, int cin, int cout, int OH, int OW, int k);
int pcx_conv2d(int mode, int precision, int B, int cin, int cout, int IH, int IW, int OH, int OW, int k, int stride,
               int pad, const float* x, const float* w, const float* dy, float* out, int accumulate, void* ws,
               size_t ws_bytes, hipStream_t stream);

void* pcx_net_create(const pcx_net_config* cfg, int64_t B, int64_t F, int64_t T);
void pcx_net_destroy(void* plan);
size_t pcx_net_workspace_bytes(const void* plan);
int pcx_net_info(const void* plan, int* nparams, int* nbn, int* ndrop, int* drop_channels);
/* byte range of a named intermediate inside the workspace (introspection / tests) */
int pcx_net_region(const void* plan, const char* name, size_t* offset, size_t* bytes);
int pcx_net_forward(const void* plan, const float* const* params, float* const* bn_stats,
                    int64_t* const* bn_counts, const float* x, const float* const* dropout,
                    int train, float* emb, void* workspace, size_t workspace_bytes,
                    hipStream_t stream);
int pcx_net_backward(const void* plan, const float* const* params, const float* x,
                     const float* const* dropout, const float* emb, const float* d_emb,
                     float* const* grads, void* workspace, size_t workspace_bytes,
                     hipStream_t stream);

/* Per-launch timing of a plan's kernels with HIP events on the launch stream.
 * pcx_net_profile(plan, 1) starts recording (and clears), pcx_net_profile_read() waits for the
 * recorded events, returns the number of distinct kernel labels and fills '\n'-separated labels,
 * total milliseconds and launch counts per label, then clears. */
int pcx_net_profile(void* plan, int enable);
/* Restrict the recording to one kernel label (e.g. "wgbd_L2"; NULL or "": every label): a timed
 * region then carries one event pair per launch of that kernel instead of one per launch. */
int pcx_net_profile_only(void* plan, const char* label);
int pcx_net_profile_read(void* plan, char* labels, size_t labels_len, float* total_ms,
                         int* counts, int max_entries);

/* Gradient buckets for a data-parallel all-reduce that overlaps the backward (DDP).
 * pcx_net_grad_buckets(plan, n, first_param) splits the parameter list into n buckets: bucket k
 * holds parameters [first_param[k], first_param[k-1]) (first_param[-1] = nparams; the list must
 * be strictly decreasing, first_param[n-1] = 0: bucket 0 holds the LAST parameters, whose
 * gradients the backward finishes first).  During every later pcx_net_backward the plan records
 * an event on its stream as soon as all gradients of a bucket are written.  pcx_net_bucket_wait
 * makes `stream` wait for bucket k's event of the most recent backward (the caller then enqueues
 * that bucket's collective on `stream`).  pcx_net_grad_stages lists the parameter indices at which
 * the backward completes a stage (descending; a good bucket boundary), returns their count.
 * n = 0 removes the buckets. */
int pcx_net_grad_buckets(void* plan, int n, const int* first_param);
int pcx_net_bucket_wait(void* plan, int k, hipStream_t stream);
int pcx_net_grad_stages(const void* plan, int* first_param, int max_entries);

/* Dropout2d keep-scale masks: out[i] = (u_i >= p) ? 1/(1-p) : 0 with u_i a counter-based
 * uniform draw from (seed, offset + i).  Not bit-compatible with torch's CPU generator. */
int pcx_dropout_masks(float* out, int64_t n, float p, uint64_t seed, uint64_t offset,
                      hipStream_t stream);

/* HBM streaming probe: dst = src (16-byte aligned, bytes % 16 == 0) with 16-byte nontemporal loads and
 * stores; the achievable copy rate bench.py's measured_peaks reports (no reference counterpart). */
int pcx_stream_copy(const void* src, void* dst, size_t bytes, hipStream_t stream);

/* ------------------------------------------------------------------ feature path
 * Replaces torchaudio.transforms.MFCC / MelSpectrogram + AmplitudeToDB as called by
 * MFCCExtractor / MelSpectrogramExtractor (src/datasets/features.py:22-150), the random gain of
 * PhonemeContrastiveDataset._augment_waveform (src/datasets/dataset.py:147-172) and the
 * TimeMask / FrequencyMask / GaussianNoise transforms (src/datasets/transforms.py:25-97).
 *
 * pcx_melspec: wave [n][S] fp32, gain [n] or NULL -> mel [n][n_mels][T] (T = 1 + S / hop; periodic
 * hann, center=True reflect padding, power 2) and tile_max [n][ceil(T/32)].  fb is the HTK mel
 * filterbank [n_freq][n_mels] zero-padded to [fb_rows = ceil((n_fft/2+1)/32)*32][fb_cols =
 * ceil(n_mels/32)*32].  n_fft/2+1 <= 256, n <= 65535 per call.
 * pcx_mel_finish: dB = 10 log10(max(mel, 1e-10)), floored at (max over a group of clamp_group
 * consecutive clips) - top_db when top_db > 0; then out[v][k][t] = sum_m dct[m][k] dB[m][t]
 * (dct [n_mels][n_out], DCT-II ortho) or, dct == NULL, out = dB.  gmax_ws: ceil(n/clamp_group)
 * floats.  out view stride out_stride >= n_out * T (room for delta features after the block).
 * pcx_compute_deltas: ComputeDeltas(win_length=5, mode="replicate") of [n][F][T] blocks.
 * pcx_specaug: in place on x [n][F][T]: t in [tband[2v], tband[2v+1]) or f in [fband[2v],
 * fband[2v+1]) -> 0 (bands may be NULL), then + level[v] * noise (noise [n][F][T] given, or drawn
 * from N(0,1) by a counter-based generator keyed by seed when noise == NULL). */
int pcx_melspec(const float* wave, int64_t n, int64_t S, const float* gain, const float* fb, int n_fft,
                int hop, int n_mels, int fb_rows, int fb_cols, float* mel, float* tile_max,
                hipStream_t stream);
int pcx_mel_finish(const float* mel, const float* tile_max, int64_t n, int64_t T, int n_mels,
                   int clamp_group, float top_db, const float* dct, int n_out, float* gmax_ws,
                   float* out, int64_t out_stride, hipStream_t stream);
int pcx_compute_deltas(const float* in, int64_t in_stride, float* out, int64_t out_stride, int64_t n,
                       int F, int64_t T, hipStream_t stream);
int pcx_specaug(float* x, int64_t n, int F, int64_t T, const int* tband, const int* fband,
                const float* level, const float* noise, uint64_t seed, hipStream_t stream);

/* Host-side (no GPU) reproduction of the reference's per-view random draws, bit-exact with
 * Python's `random` and torch's CPU generator as the reference calls them: for view v,
 * gain[v] from seed gain_seeds[v] (dataset.py:147-172) and, from aug_seeds[v] (+1000 per enabled
 * transform, transforms.py:139-143), the time band, frequency band ([start, end), {0, 0} when
 * not drawn) and the noise level (0 when not drawn).  Either seed array may be NULL. */
typedef struct pcx_aug_config {  /* probabilities and bounds are doubles, as the Python floats */
    int time_enabled, time_width;
    double time_prob;
    int freq_enabled, freq_width;
    double freq_prob;
    int noise_enabled;
    double noise_min, noise_max, noise_prob;
} pcx_aug_config;
int pcx_draw_view_params(const int64_t* gain_seeds, const int64_t* aug_seeds, int64_t n, int F, int T,
                         const pcx_aug_config* cfg, float* gain, int* tband, int* fband, float* level);

#ifdef __cplusplus
}
#endif
#endif /* PCX_H_ */
