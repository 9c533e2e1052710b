/*
 * frhip_testing.h — kernel-level entry points of libfrhip for parity tests.
 *
 * Not part of the drop-in surface (include/frhip.h): these expose single
 * kernels so tests can compare each against a PyTorch-CPU fp32 op of the same
 * shape (one Conv2d of net.BasicBlockIR, the stem, the matcher's top-k).
 * All pointers are device pointers; every call is asynchronous on `stream`.
 */
#ifndef FRHIP_TESTING_H_
#define FRHIP_TESTING_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* y = epi(conv(pre(x))) in NHWC f32, w [cout][kh][kw][cin].
 * epi: 0 affine, 1 affine+PReLU, 2 affine+residual(res same shape as y),
 *      3 affine+residual(res[b][2oy][2ox], res spatial res_h x res_w), 4 raw.
 * pre_scale/pre_shift may be NULL (no pre-affine).  nsplit > 1 only with epi 4:
 * y then holds nsplit partial slabs of B*Ho*Wo*cout floats.
 * tile: 0 = 256x64, 1 = 128x128, 2 = 128x64, 3 = 64x128, 4 = 256x128, 5 = 128x256.
 * stream_k: 1 = persistent stream-K schedule (nsplit must be 1), 0 = one block per tile.
 * precision: 0 = f32 MFMA, 1 = bf16x3 split (tiles 1, 3, 4, 6, 7, 8 only). */
int frt_conv2d(const float* x, const float* w, float* y, int B, int H, int W, int cin, int cout, int kh, int kw,
               int stride, int pad, const float* pre_scale, const float* pre_shift, const float* post_scale,
               const float* post_shift, const float* prelu, const float* res, int res_h, int res_w, int epi,
               int nsplit, int tile, int stream_k, int precision, void* stream);

/* Winograd F(2x2,3x3) stride-1 pad-1 conv (the FR_CONV_WINOGRAD path): same tensors as
 * frt_conv2d with kh = kw = 3; w is the untransformed [cout][3][3][cin] filter (transformed
 * into a scratch buffer here).  epi: 1 (needs pre) or 2 (no pre).  cin, cout % 32 == 0.
 * Synchronises. */
int frt_conv2d_winograd(const float* x, const float* w, float* y, int B, int H, int W, int cin, int cout,
                        const float* pre_scale, const float* pre_shift, const float* post_scale,
                        const float* post_shift, const float* prelu, const float* res, int epi, void* stream);
/* Winograd F(4x4,3x3) (the FR_CONV_WINOGRAD4 path, conv_winograd4.hip), same arguments;
 * cin % 16 == 0, cout % 16 == 0; epi also 0 (affine) and 5 (affine + residual + PReLU), and 1 without
 * pre-BN (the detector's convs).  frt_conv2d_winograd4 gives launch_wino4 a split-K workspace
 * (small grids then split the K loop over items + a reduce pass) unless frt_set_wino4_split(0). */
int frt_set_wino4_split(int on);
/* A/B (process-wide): the ConvTile of the fused stride-2 conv2 + conv-shortcut launches of
 * non-serving batches (-1: the built-in rule).  Forwards already captured in graphs keep theirs. */
int frt_set_conv2sc_tile(int tile);
/* A/B (process-wide): tile blocks per XCD item group of the F(4x4) launches (0: the built-in rule,
 * 32 items per group; 8 x 8 at 512 channels).  Forwards already captured in graphs keep theirs. */
int frt_set_wino4_nbg(int nbg);
/* A/B (process-wide, default 1): item shapes of whole-item F(4x4) launches without pre-BN.  A layer
 * of 65..96 output channels (the detector's 80/88-channel convs) runs items of 16 tiles x 96 couts
 * (six MFMA waves, two transform waves) instead of two 64-cout items; one of at most 32 (the
 * detector's stem conv and head outputs) items of 32 tiles x 32 couts instead of 64-cout items
 * with two idle MFMA waves.  mode 1: when the 64-cout items take more than one round of
 * workgroups; 2: at every grid size (tests); 0: never.  Graphs captured before keep theirs. */
int frt_set_wino4_shapes(int mode);
/* At most s K parts per item when a small F(4x4) grid runs split-K (0 = no cap; graphs captured
 * before the call keep their schedule). */
int frt_set_wino4_max_split(int s);
/* Poll bound of wino4_kernel's ring hand-off waits (default 65536; n < 0 restores it, 0 makes
 * every wait that does not find its step ready at once expire).  An expired wait stores an error
 * code into the launch's host-pinned error word: handle calls then fail with FR_ERR_HIP ("F(4x4)
 * ring hand-off timed out") -- fr_embed_host / fr_match_topk_host / fr_detect / fr_profile_read
 * after their sync, the asynchronous calls at their next entry -- and frt_conv2d_winograd4 after
 * its sync.  Applies to launches issued after the call (captured graphs keep theirs). */
int frt_set_wino4_poll_limit(int n);
/* The stage-1 stride-2 conv2 (64 -> 64, MaxPool2d(1,2) shortcut) of batches >= 16 on its band
 * kernel (conv_s2.hip, on = 1, default) or on the implicit-GEMM kernel (0).  Handles issue the
 * choice at launch time; graphs captured before the call keep theirs. */
int frt_set_s2_band(int on);
/* The band kernel alone: y [B][H/2][W/2][64] = conv3x3 s2 p1 (x [B][H][W][64], w [64][3][3][64])
 * * post_scale + post_shift + res[b][2oy][2ox] (res [B][H][W][64]); even H, W in [16, 112].
 * Asynchronous on stream. */
int frt_conv2d_s2band(const float* x, const float* w, float* y, int B, int H, int W, const float* post_scale,
                      const float* post_shift, const float* res, void* stream);
/* Handle h runs every body 3x3 conv of forwards of n <= max_n crops (default 2; 0 = never) on the
 * serving-batch kernel (conv_small.hip: one launch per layer, 16 pixels x 16 couts per workgroup
 * with the whole K reduction inside it) instead of F(4x4) split-K + fixup and the split-K direct
 * convs.  Drops captured graphs. */
int frt_set_small_conv(fr_handle* h, int max_n);
/* Output-pixel limit (n * Ho * Wo) of a batch-1 layer on the serving kernel (default 4,096:
 * stage 1's 56x56 layers join stages 2-4; 1,024 keeps them on F(4x4) split-K).  A/B only. */
int frt_set_small_conv_pixels(fr_handle* h, int max_m1);
/* A/B switch (default on): in a one-lane forward, a body conv2 on the serving kernel also writes
 * BN(y) for the next block's conv1 (its pre-activation BN), which then runs without pre-BN. */
int frt_set_small_conv_pre_epilogue(fr_handle* h, int on);
/* A/B switch (default on): in a forward the serving kernel does not take (n > 2 crops),
 * activations passed between two F(4x4) layers are stored channel-blocked ([n][C/16][H][W][16])
 * instead of NHWC (bitwise the same embeddings). */
int frt_set_wino4_blocked(fr_handle* h, int on);
/* A/B switch (default on): in a one-lane forward, activations passed between two layers on the
 * serving kernel are stored channel-blocked ([n][C/16][H][W][16]) instead of NHWC. */
int frt_set_small_conv_blocked(fr_handle* h, int on);
/* The serving-batch kernel alone: y = epi(conv3x3 pad 1 stride s (x) [+ conv1x1 stride s (x2)
 * against weight columns 9*cin .. + cin2]), w [cout][9*cin + cin2]; pre-BN only with epi 1;
 * epi 0, 1, 2 (res shaped like y) or 3 (res [B][H][W][cout], read at (s oy, s ox)).
 * cin, cout, cin2 % 16 == 0.  Synchronises the stream before it returns (it frees the
 * temporary fragment-order copy of w it launched with). */
int frt_conv2d_small(const float* x, const float* x2, const float* w, float* y, int B, int H, int W, int cin,
                     int cin2, int cout, int stride, const float* pre_scale, const float* pre_shift,
                     const float* post_scale, const float* post_shift, const float* prelu, const float* res, int epi,
                     void* stream);
/* Handle h runs the stride-2 conv2 of a block with a conv shortcut and that shortcut as one
 * GEMM (on = 1, default: BN scales folded into the weights, extra K-steps over the block input)
 * or as two launches (0).  Drops captured graphs. */
int frt_set_fuse_shortcut(fr_handle* h, int on);
int frt_conv2d_winograd4(const float* x, const float* w, float* y, int B, int H, int W, int cin, int cout,
                         const float* pre_scale, const float* pre_shift, const float* post_scale,
                         const float* post_shift, const float* prelu, const float* res, int epi, void* stream);

/* Fused preprocess + input_layer on uint8 RGB [B][112][112][3]; w27x64 is the
 * repacked [ky][kx][c_rgb][64] weight; lut the 256-entry normalisation table. */
int frt_stem(const uint8_t* img, int B, const float* lut, const float* w27x64, const float* bn_scale,
             const float* bn_shift, const float* prelu, float* y, void* stream);

/* The host similarity fit of fr_align_faces: src/dst float [n][2] -> M double [2][3]. */
int frt_fit_similarity(const float* src, const float* dst, int n, double* M);

/* The detector stem's MaxPool2d(3, 2, 1) alone: x [B][H][W][C] -> y [B][(H+1)/2][(W+1)/2][C], NHWC
 * f32, C % 4 == 0, 16-byte aligned.  Asynchronous on stream. */
int frt_maxpool3(const float* x, int B, int H, int W, int C, float* y, void* stream);

/* Row-wise top-k of a [n][G] score matrix (score desc, equal scores by descending index; k in [1, G]). */
int frt_topk(const float* scores, int n, int G, int k, int32_t* idx, float* val, void* stream);

/* Detector internals of fr_detect for n <= max_frames frames: letterbox + network only.
 * heads: device f32, the three levels' maps back to back, each [n][H/s][W/s][32] for
 * s = 8, 16, 32 (channels: cls a0, cls a1 logits | bbox a0 (4), a1 (4) | kps a0 (10), a1 (10)
 * in stride units | 2 zero pads); canvas: device uint8 [n][640][640][3] letterboxed frames,
 * or NULL.  Synchronises. */
int frt_detector_forward(fr_handle* h, const uint8_t* frames, int n, int height, int width, float* heads,
                         uint8_t* canvas, void* stream);
/* A/B: the stem and stage 1 skip the letterbox's invariant bottom rows (on, the default) or run
 * the full 640-row canvas (0).  Both compute the same network to fp32 rounding. */
int frt_set_detector_row_reduction(fr_handle* h, int on);

#ifdef __cplusplus
}
#endif
#endif /* FRHIP_TESTING_H_ */
