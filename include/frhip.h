/*
 * frhip.h — C ABI of the MI355X (gfx950) face embed + match hot path.
 *
 * The reference (tuoasty/FaceRecognitionPipeline) has no FFI: its seams are
 * Python duck types.  Each entry point below replaces one
 * of them; the Python host layer (facerecognitionpipeline_amd/face_embedder.py,
 * gallery_manager.py) binds these symbols with ctypes and keeps the
 * reference's method names, argument meaning and exception types.
 *
 * Conventions
 *  - Return value: FR_OK (0) or a negative FR_ERR_* code; fr_last_error()
 *    gives the message.  No call aborts the process.
 *  - "device" pointers are HIP device allocations on the handle's device;
 *    "host" pointers are ordinary host memory, borrowed for the call only.
 *  - `stream` is a hipStream_t (NULL = the null stream).  Device-pointer calls
 *    are asynchronous on that stream; host-pointer calls synchronise.  Every call
 *    on one handle must use the SAME stream: the handle's workspace (activations,
 *    stream-K slabs and tickets, staging buffers, captured graphs) is shared by
 *    all of its calls and only stream order keeps them apart.
 *  - Device-side errors: a kernel that detects a broken invariant (wino4_kernel: an LDS ring
 *    hand-off that timed out) records it in the handle's error word instead of hanging the GPU.
 *    Calls that synchronise (fr_embed_host, fr_match_topk_host, fr_detect, fr_blur_scores,
 *    fr_profile_read) then return FR_ERR_HIP for their own work; asynchronous calls (fr_embed,
 *    fr_embed_match, fr_match_topk) return it at their next entry once the faulty work has
 *    completed.  Results of the work queued before such an error are invalid.
 *  - One mutex per handle: a handle may be shared by threads (the reference
 *    server shares one FaceEmbedder/GalleryManager across Flask request
 *    threads, face_recognition_server.py:1102).
 *  - Embeddings are 512-d float32 rows; images are uint8 RGB HWC, C-contiguous:
 *    112x112x3 (the reference's aligned crops, face_recognition.py:64-74), or any
 *    size for fr_embed / fr_embed_host, which resize it first (face_embedder.py:94-96).
 */
#ifndef FRHIP_H_
#define FRHIP_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FR_OK 0
#define FR_ERR_INVALID_ARGUMENT (-1) /* Python: ValueError  */
#define FR_ERR_MISSING_PARAM (-2)    /* Python: RuntimeError (load_state_dict strict) */
#define FR_ERR_HIP (-3)              /* Python: RuntimeError */
#define FR_ERR_STATE (-4)            /* Python: RuntimeError (not finalised / no gallery) */
#define FR_ERR_UNSUPPORTED (-5)      /* Python: NotImplementedError */

#define FR_EMBED_DIM 512
#define FR_INPUT_SIZE 112

typedef struct fr_handle fr_handle;

/* Build an empty model.  Replaces FaceEmbedder.__init__'s
 * `net.build_model(architecture)` (face_embedder.py:27-49).
 * architecture: "ir_50" | "ir_101" (also "ir_18", "ir_34"); model_type: "adaface" (AdaFace
 * net.py keys) or "arcface" (the insightface arcface_torch IResNet behind the reference's ONNX
 * files, face_embedder.py:64-88: (x-127.5)/127.5 input, conv downsample in every stage, affine
 * BN1d, no L2 inside the model; keys conv1, bn1, prelu, layerS.U.{bn1,conv1,...}, bn2, fc, features).
 * max_batch: images per internal forward chunk (workspace sizing), 1..512. */
int fr_create(const char* architecture, const char* model_type, int device, int max_batch, fr_handle** out);
int fr_destroy(fr_handle* h);

/* One state-dict tensor (AdaFace: key WITHOUT the "model." prefix), float32
 * host data in PyTorch's layout (conv weights [out][in][kh][kw]).  Replaces
 * `self.model.load_state_dict(model_statedict)` (face_embedder.py:51-53);
 * num_batches_tracked keys are accepted and ignored. */
int fr_set_param(fr_handle* h, const char* name, const float* host_data, int64_t numel);
/* Fold BatchNorms, repack weights NHWC, upload.  Missing keys -> FR_ERR_MISSING_PARAM
 * (strict load_state_dict semantics).  Replaces `.to(device).eval()` (face_embedder.py:55-56). */
int fr_finalize(fr_handle* h);

/* Embed n crops.  Replaces FaceEmbedder.extract_embeddings_batch
 * (face_embedder.py:137-182) and extract_embedding (:112-135): cv2.resize to 112x112
 * (INTER_LINEAR, OpenCV fixed point) when height x width is not 112x112 (:94-96), BGR + LUT
 * normalise, IR forward, x/||x||, and with normalize!=0 the extra e/(||e||+1e-8).
 * rgb: device [n][height][width][3] uint8 (1 <= height, width <= 8192); out: device [n][512]. */
int fr_embed(fr_handle* h, const uint8_t* rgb, int n, int height, int width, float* out, int normalize,
             void* stream);
/* Same with host buffers (H2D, forward, D2H, synchronise). */
int fr_embed_host(fr_handle* h, const uint8_t* rgb, int n, int height, int width, float* out, int normalize);
/* The resize step alone: dst[i] = cv2.resize(src[i], (112, 112), INTER_LINEAR) for n device crops
 * of height x width (face_embedder.py:94-96).  src: device [n][height][width][3] uint8; dst: device
 * [n][112][112][3] uint8. */
int fr_resize_crops(fr_handle* h, const uint8_t* src, int n, int height, int width, uint8_t* dst, void* stream);

/* Replace the gallery matrix (G rows of D=512 float32).  Replaces the per-query
 * `np.vstack` of GalleryManager.get_gallery_embeddings (gallery_manager.py:177-187):
 * the handle keeps one device-resident copy until the next fr_gallery_set.
 * src_is_device: 1 if E is a device pointer.  G == 0 clears the gallery. */
int fr_gallery_set(fr_handle* h, const float* E, int G, int D, int src_is_device, void* stream);
int fr_gallery_size(fr_handle* h, int* G);
/* Incremental gallery maintenance, so an enrollment change does not re-upload (or, across
 * GPUs, re-broadcast) the whole matrix.  Rows are in get_gallery_embeddings order (dict
 * insertion order, gallery_manager.py:177-187).
 * write_rows: rows [row0, row0+n) := E (row0 <= G; rows past G extend the gallery) -- add_student
 *   appends (:71-102), add_student(overwrite=True) / update_embeddings rewrite in place (:124-158).
 * delete_rows: drop rows [row0, row0+n), later rows move up -- delete_student (:160-169).
 * read: copy rows out (host or device). */
int fr_gallery_write_rows(fr_handle* h, int row0, int n, const float* E, int src_is_device, void* stream);
int fr_gallery_delete_rows(fr_handle* h, int row0, int n, void* stream);
int fr_gallery_read(fr_handle* h, int row0, int n, float* out, int dst_is_device, void* stream);

/* GalleryManager._aggregate_embeddings (gallery_manager.py:297-317) incl. the quality
 * filter (:104-122) for n_students at once (bulk enrollment).  emb: device [total][512] f32,
 * student i = rows [offsets[i], offsets[i+1]) (host offsets, offsets[0] = 0, 1..1024 rows
 * each); templates: device [n_students][512]; kept: device [n_students] rows surviving the
 * filter, or NULL.  Synchronises. */
#define FR_TEMPLATE_MEAN 0
#define FR_TEMPLATE_MEDIAN 1
#define FR_TEMPLATE_WEIGHTED_MEAN 2
int fr_build_templates(fr_handle* h, const float* emb, const int32_t* offsets, int n_students, int method,
                       float min_similarity, float* templates, int32_t* kept, void* stream);

/* Batched GalleryManager.search (gallery_manager.py:189-205): q/(||q||+1e-8),
 * S = E.q (fp32), top-k by descending score; equal scores by DESCENDING gallery row (a stable
 * ascending argsort reversed, which is what the reference's np.argsort(S)[::-1] gives; DESIGN.md
 * §3 "Tie policy").  k must be in [1, G] (G = fr_gallery_size), else FR_ERR_INVALID_ARGUMENT:
 * the Python layer clamps top_k to G as search() does.
 * Q: device [n][512]; idx: device [n][k] int32 gallery rows; score: device [n][k]. */
int fr_match_topk(fr_handle* h, const float* Q, int n, int k, int32_t* idx, float* score, void* stream);
/* Host-buffer variant (synchronises). */
int fr_match_topk_host(fr_handle* h, const float* Q, int n, int k, int32_t* idx, float* score);

/* Fused unit of work of FaceMatcher.match_single_face (face_matcher.py:52-58),
 * batched: embed(normalize=1) then match (same k contract and tie policy as fr_match_topk).
 * emb_out may be NULL.  Device pointers. */
int fr_embed_match(fr_handle* h, const uint8_t* rgb, int n, int k, int32_t* idx, float* score, float* emb_out,
                   void* stream);

/* FaceAligner.align for n faces of one frame (face_recognition.py:50-75): similarity fit of
 * each face's 5 landmarks to the reference template (cv2.estimateAffinePartial2D semantics,
 * host, double) then warpAffine INTER_LINEAR / BORDER_CONSTANT 0 on the device, so the crops
 * stay in HBM for fr_embed.  frame: device uint8 [height][width][3] RGB; landmarks: host float
 * [n][5][2]; out: device uint8 [n][out_size][out_size][3]; tforms: host double [n][2][3] forward
 * maps as cv2 returns them, or NULL.  Synchronises (the maps are staged from the host). */
int fr_align_faces(fr_handle* h, const uint8_t* frame, int height, int width, const float* landmarks, int n,
                   int out_size, uint8_t* out, double* tforms, void* stream);
/* cv2.warpAffine(frame, M, (out_size, out_size), INTER_LINEAR, BORDER_CONSTANT, 0) for n
 * caller-supplied FORWARD maps (host double [n][2][3], e.g. cv2.getAffineTransform's for
 * FaceAligner.align(method != 'similarity'), face_recognition.py:66-67).  Synchronises. */
int fr_warp_affine(fr_handle* h, const uint8_t* frame, int height, int width, const double* tforms, int n,
                   int out_size, uint8_t* out, void* stream);
/* FaceQualityFilter.compute_blur_score for n images of one size (face_recognition.py:94-99):
 * cv2.Laplacian(gray, CV_64F).var() with gray = cvtColor(RGB2GRAY) of a 3- (or 4-) channel
 * image, or the image itself for channels == 1 (the reference's 2-D branch); ksize 1,
 * BORDER_REFLECT_101.  The variance is summed in numpy's order (ndarray.var's chunked pairwise
 * sum; derived for and checked against numpy 2.2), so it is bitwise the reference's value there.
 * crops: device uint8 [n][height][width][channels], any height, width >= 1 (height * width
 * < 2^31); channels 1, 3 or 4; scores: host double [n].  Runs on `stream` (NULL: the null stream)
 * and synchronises that stream only. */
int fr_blur_scores(fr_handle* h, const uint8_t* crops, int n, int height, int width, int channels, double* scores,
                   void* stream);

/* FaceDetector.detect (face_recognition.py:31-48: insightface SCRFD det_10g at det_size
 * 640x640, det_thresh, NMS IoU 0.4) for n frames of one size.  The handle is created with
 * fr_create("scrfd_10g", "scrfd", device, max_frames (1..64), &h) and loaded with the
 * state dict of oracle/scrfd.py's network (fr_set_param / fr_finalize).
 * frames: device uint8 [n][height][width][3] RGB.  Per frame f, counts[f] = detections
 * after NMS (score order) and dets[f][i][0..14] = x1 y1 x2 y2 score, then 5 landmarks
 * (x, y), in frame pixels, for i < min(counts[f], max_faces) (host buffers; synchronises).
 * More than 4096 anchors above det_thresh in one frame -> FR_ERR_UNSUPPORTED. */
int fr_detect(fr_handle* h, const uint8_t* frames, int n, int height, int width, float det_thresh, int max_faces,
              float* dets, int32_t* counts, void* stream);

/* Conv arithmetic of this handle.  FR_PRECISION_F32 (default): exact f32 products and f32
 * accumulation on fp32 MFMA -- the parity path.  FR_PRECISION_BF16X3 (opt-in fast mode):
 * each f32 operand split into bf16 hi + lo, x.y ~= hi.hi + hi.lo + lo.hi on bf16 MFMA with f32
 * accumulation (per-product relative error ~2^-16; measured score drift in DESIGN.md). */
#define FR_PRECISION_F32 0
#define FR_PRECISION_BF16X3 1
int fr_set_precision(fr_handle* h, int mode);

/* Algorithm of the stride-1 3x3 convs (the bulk of the network's MACs).  All compute in f32.
 * FR_CONV_WINOGRAD4 (default): Winograd F(4x4,3x3) -- 36 f32-MFMA products per 4x4 tile
 * instead of 144, filters transformed once (on selection / at fr_finalize), pre-BN folded
 * into them; embeddings within 1e-5 of the CPU reference (tests).  FR_CONV_WINOGRAD:
 * F(2x2,3x3), 16 products per 2x2 tile instead of 36.  FR_CONV_DIRECT: the implicit-GEMM
 * kernel for every conv.  FR_PRECISION_BF16X3 runs the direct split-bf16 kernel. */
#define FR_CONV_DIRECT 0
#define FR_CONV_WINOGRAD 1
#define FR_CONV_WINOGRAD4 2
int fr_set_conv_algorithm(fr_handle* h, int algo);

/* hipGraph replay of small forwards.  With max_n > 0 (<= max_batch), every embed of n <= max_n
 * crops (fr_embed, fr_embed_host, fr_embed_match) runs its ~100 kernel launches as one captured
 * graph: the first call for an n runs eagerly and captures, later calls replay (same kernels and
 * arguments, so bit-identical results).  0 (default) disables; changing the precision, the conv
 * algorithm or the weights drops the captured graphs.  fr_graph_count reports how many exist. */
int fr_set_graph_batch(fr_handle* h, int max_n);

/* Lanes of a large forward.  With min_n > 0, a forward of n crops runs as
 * min(max_lanes, n / min_n) concurrent parts of near-equal size (n < 2 * min_n: one part;
 * max_lanes in [1, 4]): the first
 * part on the call's stream, the others on internal streams forked from it and joined back
 * before the call returns, each with its own activation and split-K workspace (allocated on first
 * use, ~1 GB per extra lane of 64 crops).  Launches alternate between the parts, so the last,
 * part-empty round of one part's layer runs beside another part's launch of the same layer.
 * Embeddings are those of separate forwards of the parts (batch-invariant to ~1e-6).
 * min_n 0 = one lane.  fr_create's default: FR_LANES_MIN_DEFAULT crops per lane, at most
 * FR_LANES_MAX_DEFAULT lanes (measured on MI355X, IR-101 C3: batch 256 as 2 x 128 +6%, as 3 or 4
 * parts -1..-2%; batch 128 as 2 x 64 +8%; batch 64 as 2 x 32 -6%).  Lane 1's workspace (~1.7 GB
 * at max_batch 256: 1.23 GB of activations for 128 crops, 0.27 GB of stream-K slabs, the
 * shortcut, split-K and head-partial buffers) is allocated by the first forward that uses it; if that allocation fails the
 * forward runs as one lane and lanes stay off until the next fr_set_lanes. */
#define FR_LANES_MIN_DEFAULT 64
#define FR_LANES_MAX_DEFAULT 2
int fr_set_lanes(fr_handle* h, int min_n, int max_lanes);
/* The lane setting in force: min_n is 0 after a failed lane-workspace allocation turned lanes off,
 * and fell_back is then 1 (until the next fr_set_lanes).  Any output pointer may be NULL. */
int fr_get_lanes(fr_handle* h, int* min_n, int* max_lanes, int* fell_back);
int fr_graph_count(fr_handle* h, int* count);

/* Per-kernel-class timing with HIP events on the call stream (bench roofline).
 * enable=1 starts recording; fr_profile_read synchronises and returns, since the
 * last read: summed milliseconds and algorithmic FLOPs of the conv launches (direct and
 * Winograd), their launch count, and the summed milliseconds of all launches. */
int fr_profile_enable(fr_handle* h, int enable);
int fr_profile_read(fr_handle* h, double* conv_ms, double* conv_flop, int64_t* conv_launches, double* total_ms);
/* Breakdown of the last fr_profile_read by kernel class: summed ms, algorithmic (direct-conv)
 * FLOPs, FLOPs the MFMA pipe executed (F(4x4,3x3), the default: 36 products per 4x4 canvas tile
 * instead of the direct conv's 144; F(2x2,3x3): 16 per 2x2 tile instead of 36) and launch count. */
#define FR_PROF_OTHER 0
#define FR_PROF_CONV_DIRECT 1
#define FR_PROF_CONV_WINOGRAD 2
int fr_profile_kernel(fr_handle* h, int kind, double* ms, double* flop, double* exec_flop, int64_t* launches);

/* Last error message of this handle (or of the last failed fr_create if h is NULL). */
const char* fr_last_error(fr_handle* h);
/* Library build/version string; it ends in "build <id>", the content hash of every source and
 * flag the library was built from (build.py build_id), which profiles are stamped with. */
const char* fr_version(void);

#ifdef __cplusplus
}
#endif
#endif /* FRHIP_H_ */
