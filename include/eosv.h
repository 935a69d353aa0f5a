/*
 * eosv.h -- C ABI of the MI355X-native clip-embedding + one-shot matching path.
 *
 * The reference (lovelyqian/Embodied-One-Shot-Video-Recognition) is pure Python with
 * no FFI; its hot path is implicit torch/cuDNN work behind three Python call sites.
 * Each entry point below replaces one of them (reference file:line in the comment);
 * the Python drop-in modules (models.py, network_test.py, classifier.py, ...) bind
 * these with ctypes.
 *
 * Conventions:
 *   - every function returns 0 (EOSV_OK) or a negative eosv_status; a thread-local
 *     message is available from eosv_last_error().  No exception crosses the ABI.
 *   - all d_* pointers are DEVICE pointers owned by the caller; nothing is freed
 *     across the boundary.  The library owns weights + workspace inside the handle.
 *   - calls enqueue on the given stream (a hipStream_t; NULL = default stream) and do
 *     not synchronise.  A handle is bound to one device and is not re-entrant.
 */
#ifndef EOSV_H
#define EOSV_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ihipStream_t* eosv_stream_t; /* == hipStream_t */
typedef struct eosv_handle eosv_handle;

typedef enum {
  EOSV_OK = 0,
  EOSV_ERR_ARG = -1,         /* bad argument / shape / missing tensor */
  EOSV_ERR_HIP = -2,         /* a HIP runtime call failed */
  EOSV_ERR_OOM = -3,         /* device allocation failed */
  EOSV_ERR_UNSUPPORTED = -4, /* arch / dtype / shape not implemented */
  EOSV_ERR_STATE = -5        /* e.g. forward before eosv_load_weights */
} eosv_status;

typedef enum { EOSV_ARCH_R18 = 18, EOSV_ARCH_R50 = 50, EOSV_ARCH_R101 = 101 } eosv_arch;
/* EOSV_F32X3: f32-accurate split-bf16 arithmetic.  Activations are stored as bf16 (hi, lo)
 * pairs (hi = bf16(v), lo = bf16(v - hi): 16 significant bits), weights likewise, and every
 * conv sums the three bf16 MFMA products hi.hi + lo.hi + hi.lo in f32 ("bf16x3"): ~2^-16
 * relative per product, against 2^-8 for plain bf16.  The fused stem + maxpool uses the same
 * split (frames and weights as hi + lo, three bf16 MFMAs per k-slice). */
typedef enum { EOSV_F32 = 0, EOSV_BF16 = 1, EOSV_F32X3 = 2 } eosv_dtype;
typedef enum { EOSV_MATCH_PROTONET = 0, EOSV_MATCH_COSINE = 1 } eosv_match_kind;

typedef struct {
  int arch;        /* eosv_arch */
  int dtype;       /* eosv_dtype: arithmetic of the conv stack (f32 = exact-f32 MFMA) */
  int height;      /* frame height (224, 256, ...) */
  int width;
  int max_frames;  /* frames per internal chunk; workspace is sized for this */
  int device;      /* HIP device ordinal */
  int num_classes; /* fc output size (reference: num_classes_train = 64) */
} eosv_desc;

/* Create a handle (allocates workspace).  Replaces the construction at
 * reference models.py:9-16 / 24-31 (torchvision resnet18/50 + fc). */
int eosv_create(const eosv_desc* desc, eosv_handle** out);

/* Upload a state_dict (reference keys, models.py:14-16: convnet.{0,1,4..7}.*, fc.*).
 * host_ptrs[i] points to numel[i] float32 values (num_batches_tracked entries are
 * ignored and may be NULL).  BN is folded into the conv weights here.
 * Replaces load_state_dict(torch.load(pkl)) at network_test.py:133-135. */
int eosv_load_weights(eosv_handle* h, const char* const* names, const void* const* host_ptrs,
                      const int64_t* numel, int n);

/* Backbone forward: d_frames [B,3,H,W] float32 NCHW (post-Normalize) ->
 * d_feat [B,D] float32 (D = 512 for R18, 2048 for R50/R101) = convnet(x).view(B,-1).
 * Replaces self.convnet(x) at models.py:19-20 / 34-35. */
int eosv_backbone_forward(eosv_handle* h, const float* d_frames, int B, float* d_feat,
                          eosv_stream_t stream);

/* fc head: d_feat [B,D] -> d_logits [B,num_classes].  models.py:21 / 36. */
int eosv_fc_forward(eosv_handle* h, const float* d_feat, int B, float* d_logits,
                    eosv_stream_t stream);

/* Clip embedding: for clip c, frames d_feat[offsets[c] .. offsets[c]+counts[c]) are
 * (optionally) L2-normalised (F.normalize p=2, eps 1e-12) and averaged with a
 * sequential f32 sum / count.  d_offsets/d_counts are device int32 [n_clips].
 * Replaces network_test.py:62-65 (and :79-80 with counts == 1). */
int eosv_clip_embed(const float* d_feat, const int32_t* d_offsets, const int32_t* d_counts,
                    int n_clips, int D, int l2, float* d_emb, eosv_stream_t stream);

/* Segment mean: d_feat [n_seg*seg_len, D] -> d_seg [n_seg, D] = mean over seg_len
 * consecutive rows.  network_test.py:188-189, 204-205. */
int eosv_segment_mean(const float* d_feat, int n_seg, int seg_len, int D, float* d_seg,
                      eosv_stream_t stream);

/* One-shot matching of n_episodes episodes in one launch.
 *   d_query    [n_episodes, D]      query clip embedding of each episode
 *   d_support  [sum S_e, D]         support embeddings, episode e at rows sup_off[e]..
 *   d_sup_off  [n_episodes+1]       int32 row offsets into d_support
 *   d_sup_slot [sum S_e]            int32 prototype slot of each support row
 *                                   (first-appearance order of its label, classifier.py:20-36)
 *   d_n_proto  [n_episodes]         int32 prototypes per episode (n_way <= 64; larger
 *                                   values are clamped to 64 on the device)
 * kind = PROTONET: f64 cdist to per-slot means (scipy's sequential f64 sum, no fused
 *        multiply-add: distances bit-identical to classifier.py:63 on the same features)
 *        -> f32 -> softmax(-d) -> argmax (classifier.py:43-90); d_pred = prototype position,
 *        d_score = the f32 distances (the top-2 margin of an episode is read from them).
 * kind = COSINE:   cosine similarity to every support row -> argmax (classifier.py:117-120);
 *        d_pred = support row index within the episode, d_score = similarities.
 * d_score [n_episodes, max_cols] f32 (may be NULL), max_cols = 64. */
int eosv_match(const float* d_query, const float* d_support, const int32_t* d_sup_off,
               const int32_t* d_sup_slot, const int32_t* d_n_proto, int n_episodes, int D,
               int kind, int64_t* d_pred, float* d_score, eosv_stream_t stream);

/* Config-3 gallery matching (network_test.py:207-214 + models.py:42-56):
 * dist = cdist(d_seg [S,D], d_gallery [G,D]) in f64 -> f32 -> 3-tap smoothing
 * [l1,l2,l1] along the S axis with zero padding -> first argmin over G per row.
 * d_ids [S] int64; d_dist [S,G] f32 smoothed distances (may be NULL).  One fused pass: no
 * device allocation, no [S,G] scratch (d_ids doubles as the per-row argmin accumulator). */
int eosv_segment_match(const float* d_seg, int S, const float* d_gallery, int G, int D,
                       float lamda1, float lamda2, int64_t* d_ids, float* d_dist,
                       eosv_stream_t stream);

/* The same for n_episodes independent episodes in one call (network_test.py:207-214 run per
 * episode): d_seg [n_episodes*S, D] (episode-major), one shared gallery; the smoothing never
 * crosses an episode boundary.  d_ids [n_episodes*S]; d_dist [n_episodes*S, G] or NULL. */
int eosv_segment_match_episodes(const float* d_seg, int n_episodes, int S, const float* d_gallery, int G,
                                int D, float lamda1, float lamda2, int64_t* d_ids, float* d_dist,
                                eosv_stream_t stream);

/* TemporalLayer (models.py:42-56, PyTorch-1.x conv semantics): y[r][c] = l1*x[r][c-1]
 * + l2*x[r][c] + l1*x[r][c+1] along the last axis, zero padded; d_x/d_y [rows, cols]. */
int eosv_temporal_smooth(const float* d_x, int rows, int cols, float lamda1, float lamda2,
                         float* d_y, eosv_stream_t stream);

/* Frame ingest (utils.py:80-91 test transform): d_rgb [n_frames, H, W, 3] uint8 decoded
 * frames -> centre crop `crop` -> /255 -> (x - mean[c]) / std[c] -> d_out [n_frames,3,crop,crop]
 * f32 NCHW.  mean/std are HOST arrays of 3 floats.  Bit-identical to torchvision's
 * CenterCrop + ToTensor + Normalize on the same pixels. */
int eosv_normalize_frames(const uint8_t* d_rgb, int n_frames, int H, int W, int crop, const float* mean,
                          const float* std, float* d_out, eosv_stream_t stream);

/* Same transform with an explicit window (utils.py:57-78 ClipRandomCrop + ClipRandomHorizontalFlip,
 * train mode): rows top .. top+crop-1, columns left .. left+crop-1, mirrored when flip != 0.
 * The window must lie inside H x W. */
int eosv_crop_normalize_frames(const uint8_t* d_rgb, int n_frames, int H, int W, int crop, int top, int left,
                               int flip, const float* mean, const float* std, float* d_out, eosv_stream_t stream);

/* Deterministic synthetic frames, bit-identical to eosv/synth.py:synth_frame.
 * For frame f: class seed, video seed, noise seed (u64) and frame id in d_params
 * [n_frames, 4] (u64); writes d_frames [n_frames,3,H,W] f32 NCHW.  Frames with
 * frame id 0 are written as zeros (the reference's zero padding, utils.py:250-253). */
int eosv_synth_frames(const uint64_t* d_params, int n_frames, int H, int W, float* d_frames,
                      eosv_stream_t stream);

/* Kernel timing for the roofline report: while enabled, every conv launch of the
 * handle is bracketed by HIP events on its stream (layer id = position in the plan:
 * 0 = stem, then each block's convs in order, fc last).  eosv_profile_read
 * synchronises on the recorded events and returns, per layer id < max_layers,
 * the summed milliseconds, summed algorithmic FLOPs (2 x MACs) and launch count;
 * the return value is the number of layer ids in the plan.  Enabling clears the log.
 * Switching it on / off also launches one empty marker kernel on the null stream
 * (profile_window_begin_kernel / profile_window_end_kernel), so that a rocprofv3 trace or PMC
 * pass of the same run can select exactly the window's dispatches. */
int eosv_profile_enable(eosv_handle* h, int enable);
int eosv_profile_read(eosv_handle* h, double* ms, double* flops, int64_t* launches, int max_layers);

/* Episode-plan service (host only, no device call): n_episodes n-way k-shot plans in the
 * reference's RNG order (episode_novel_dataloader.py:35-70 drawing from Python's `random`
 * seeded with random.seed(seed)); replaces the per-episode dict rebuild + random.sample calls
 * of EpisodeDataloader.get_episode (episode_novel_dataloader.py:19-80).
 * class_sizes[c] = number of videos of class c, classes in the split list's first-appearance
 * order.  Outputs: classes [E][n_way] (class ids in sampled order; support label = position),
 * query [E][2] (position of the query class, video index in that class), support
 * [E][n_way][k_shot] (video indices, class by class).  EOSV_ERR_ARG where random.sample would
 * raise (a class with fewer videos than drawn, n_way > n_classes). */
int eosv_plan_episodes(const int32_t* class_sizes, int n_classes, int n_way, int k_shot, uint64_t seed,
                       int n_episodes, int32_t* classes, int32_t* query, int32_t* support);

/* Diagnostics (SURVEY 8(c) one-frame per-layer checksums): the backbone on d_frames
 * [B,3,H,W] (1 <= B <= max_frames) up to the end of `stage` -- 0 = stem + maxpool
 * (convnet.0-3), 1..4 = layer1..layer4 (convnet.4-7) -- written to d_out as f32 NHWC
 * [B, h, w, C] (converted from bf16 or the f32x3 split layout).  Returns the f32 elements per
 * frame (h * w * C), or a negative eosv_status.  Replaces nothing on the reference's path: it
 * exposes the intermediate maps of self.convnet (models.py:19) for parity checks. */
int eosv_backbone_probe(eosv_handle* h, const float* d_frames, int B, int stage, float* d_out,
                        eosv_stream_t stream);

/* ---- Training path (reference network_train.py:52-131, epoch_dataloader.py) ----
 * TrainNetwork.finetune_model: ResNet-18/50 in train mode (batch-statistics BN), fc +
 * CrossEntropyLoss, loss.backward(), torch.optim.SGD(momentum 0.9) on convnet and fc.  The
 * Python trainer (eosv/train.py) chains these f32 kernels; activations NHWC ([P][C] rows),
 * conv weights [Cout][KH][KW][Cin].  No handle: every call is stateless on caller buffers. */

/* Row-major C[m][n] = alpha * op(A) op(B) + beta * C (op = transpose when trans_*; beta 0: C is
 * not read) on the in-tree exact-f32 MFMA GEMM (gemm_f32.hip; deterministic, no atomics).  The
 * conv GEMMs of a training step that are not the inference conv kernels' shape: the stem's
 * forward Y = Xcol W^T (models.py:19 in train mode), strided-conv input gradients dXcol = dY W,
 * 1x1 / stem weight gradients dW = dY^T Xcol (loss.backward(), network_train.py:114), and the fc
 * (logits, its weight and input gradients).  Replaced rocBLAS sgemm in r05. */
int eosv_sgemm(int trans_a, int trans_b, int m, int n, int k, float alpha, const float* d_a, int lda,
               const float* d_b, int ldb, float beta, float* d_c, int ldc, eosv_stream_t stream);
/* Weight-gradient GEMM C[m][n] = A^T B with A [k][m], B [k][n] row-major and k (the pixel count
 * P of a conv) much larger than m, n: the reduction is split into slices (one workgroup grid
 * dimension), each writing its partial tile to d_work, then summed in slice order
 * (deterministic).  work_bytes below eosv_sgemm_tn_splitk_workspace(m, n, k) runs one slice.
 * ldc must equal n. */
int64_t eosv_sgemm_tn_splitk_workspace(int m, int n, int k);
int eosv_sgemm_tn_splitk(int m, int n, int k, const float* d_a, int lda, const float* d_b, int ldb, float* d_c,
                         int ldc, float* d_work, int64_t work_bytes, eosv_stream_t stream);
/* Weight gradient of a KxK conv without the im2col buffer: dW[Cout][KH][KW][Cin] = sum over
 * output pixels of dY[p][co] * X[in(p, kh, kw)][ci] (NHWC x [N][H][W][Cin], dY [P][Cout]), an
 * implicit GEMM on exact-f32 MFMA with the pixel reduction split into slices summed in order
 * (deterministic).  EOSV_ERR_UNSUPPORTED unless Cin % 4 == 0, Cout % 64 == 0 and K % 64 == 0,
 * K = KH KW Cin; d_work: eosv_conv_wgrad_f32_workspace(...) bytes. */
int64_t eosv_conv_wgrad_f32_workspace(int N, int H, int W, int Cin, int Cout, int KH, int KW, int stride, int pad);
int eosv_conv_wgrad_f32(const float* d_x, int N, int H, int W, int Cin, const float* d_dy, int Cout, int KH, int KW,
                        int stride, int pad, float* d_dw, float* d_work, int64_t work_bytes, eosv_stream_t stream);
/* im2col of NHWC x: col[(n, oh, ow)][(kh, kw, c)], zero padding; col2im is its adjoint
 * (gather-sum, overwrites d_x). */
int eosv_im2col(const float* d_x, int N, int H, int W, int C, int KH, int KW, int stride, int pad, float* d_col,
                eosv_stream_t stream);
int eosv_col2im(const float* d_col, int N, int H, int W, int C, int KH, int KW, int stride, int pad, float* d_x,
                eosv_stream_t stream);
/* Batch norm in train mode (nn.BatchNorm2d.train(), eps, momentum): batch mean / biased variance
 * normalise, the running estimates take the unbiased variance; y = bn(x) (+ residual) (ReLU).
 * Saves mean and 1/sqrt(var + eps) for the backward.  d_mask (optional, used with relu): one byte
 * per element, 1 where y > 0, for the backward (r05).  d_work: eosv_bn_workspace_bytes(C). */
int64_t eosv_bn_workspace_bytes(int C);
int eosv_bn_train_forward(const float* d_x, int64_t P, int C, const float* d_gamma, const float* d_beta, float eps,
                          float momentum, float* d_running_mean, float* d_running_var, const float* d_residual,
                          int relu, float* d_y, uint8_t* d_mask, float* d_save_mean, float* d_save_invstd,
                          void* d_work, eosv_stream_t stream);
/* Its backward from dy = dL/dy (masked by y > 0 when relu: from d_mask when given, else from d_y):
 * dx, dgamma, dbeta; d_dres (optional) receives the masked dy, the gradient of the residual
 * branch. */
int eosv_bn_train_backward(const float* d_dy, const float* d_y, const uint8_t* d_mask, int relu, const float* d_x,
                           int64_t P, int C, const float* d_gamma, const float* d_save_mean,
                           const float* d_save_invstd, float* d_dx, float* d_dgamma, float* d_dbeta, float* d_dres,
                           void* d_work, eosv_stream_t stream);
/* Max pool 3x3 / 2, pad 1 with argmax indices (first maximum in window order, as torch CPU);
 * backward gathers dy into the argmax positions. */
int eosv_maxpool_forward(const float* d_x, int N, int H, int W, int C, float* d_y, int32_t* d_idx,
                         eosv_stream_t stream);
int eosv_maxpool_backward(const float* d_dy, const int32_t* d_idx, int N, int H, int W, int C, float* d_dx,
                          eosv_stream_t stream);
/* Average pool over HW ([N][HW][C] -> [N][C]); dx[(n, t)][c] = dy[n][c] * scale (its backward
 * with scale 1/HW, and the clip mean's over T frames, network_train.py:110). */
int eosv_avgpool_forward(const float* d_x, int N, int HW, int C, float* d_y, eosv_stream_t stream);
int eosv_broadcast_rows(const float* d_dy, int N, int T, int C, float scale, float* d_dx, eosv_stream_t stream);
/* nn.CrossEntropyLoss (mean): per-row loss terms (sum = loss) and dL/dlogits. */
int eosv_softmax_xent(const float* d_logits, const int32_t* d_labels, int B, int C, float* d_row_loss,
                      float* d_dlogits, eosv_stream_t stream);
/* y[c] (+)= sum over rows of x[r][c]; y[r][c] += bias[c]. */
int eosv_sum_rows(const float* d_x, int rows, int C, float* d_y, int accumulate, eosv_stream_t stream);
int eosv_add_bias(float* d_y, int rows, int C, const float* d_bias, eosv_stream_t stream);
/* torch.optim.SGD step (momentum, dampening 0): buf = first ? g : momentum buf + g; p -= lr buf. */
int eosv_sgd_momentum(float* d_p, const float* d_g, float* d_buf, int64_t n, float lr, float momentum, int first,
                      eosv_stream_t stream);
/* Direct f32 convolution of NHWC d_x with d_w [Cout][KH][KW][Cin] (+ bias, + residual, ReLU) on
 * the inference conv kernels (exact-f32 MFMA implicit GEMM / stage-1 row kernel): the train-mode
 * forward of every conv but the stem, and, with eosv_flip_weights' [Cin][KH][KW][Cout] weights,
 * the input gradient of the stride-1 convs.  EOSV_ERR_UNSUPPORTED unless Cin % 32 == 0. */
int eosv_conv2d_f32(const float* d_x, int N, int H, int W, int Cin, const float* d_w, int Cout, int KH, int KW,
                    int stride, int pad, const float* d_bias, const float* d_res, int relu, float* d_y, float* d_work,
                    int64_t work_bytes, eosv_stream_t stream);
/* Workspace of eosv_conv2d_f32 (d_work / work_bytes; NULL / 0 = none; 0 bytes needed = no split): a launch
 * whose grid would leave CUs idle splits its K loop over up to 8 slices of raw partial sums,
 * summed in slice order with the bias / residual / ReLU epilogue (deterministic, not bitwise
 * equal to the unsplit order). */
int64_t eosv_conv2d_f32_workspace(int N, int H, int W, int Cin, int Cout, int KH, int KW, int stride, int pad);
int eosv_flip_weights(const float* d_w, int Cout, int KH, int KW, int Cin, float* d_wf, eosv_stream_t stream);
/* y += alpha x; NCHW -> NHWC. */
int eosv_axpy(float* d_y, const float* d_x, int64_t n, float alpha, eosv_stream_t stream);
int eosv_nchw_to_nhwc(const float* d_x, int N, int C, int H, int W, float* d_y, eosv_stream_t stream);

/* Feature dimension D of the handle's backbone. */
int eosv_feature_dim(const eosv_handle* h);

/* Device bytes held by the handle (weights + workspace). */
int64_t eosv_device_bytes(const eosv_handle* h);

const char* eosv_last_error(void);
void eosv_destroy(eosv_handle* h);

#ifdef __cplusplus
}
#endif

#endif /* EOSV_H */
