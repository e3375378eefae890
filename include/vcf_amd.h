/*
 * vcf_amd.h -- C ABI of libvcf_amd.so, the MI355X (gfx950) implementation of
 * VCF's per-frame transform -> quantize hot path.
 *
 * The reference (Sistemas-Multimedia/VCF) is pure Python; its hot path is the
 * sequence of numpy/scipy calls inside src/2D-DCT.py encode_fn/decode_fn.
 * Each entry point below replaces a span of those calls and is what a
 * reference-side ctypes binding would bind:
 *
 *   vcf_dct_dz_encode  replaces src/2D-DCT.py:276-361
 *       astype(float32), pad_and_center (:187-229), -= 128 (:292),
 *       YCoCg.from_RGB (:298), DCT2D analyze_image (:303), -p weighting
 *       (:313-327), get_subbands (:333-336), deadzone quantize_fn
 *       (:343 -> src/deadzone.py:95-102), += 128 and astype(uint8) (:348,361)
 *   vcf_dct_dz_decode  replaces src/2D-DCT.py:399-466
 *       astype(int16) - 128 (:399-403), dequantize (:411 ->
 *       src/deadzone.py:107-117), get_blocks (:416), -p de-weighting
 *       (:421-435), DCT2D synthesize_image (:440), remove_padding (:444),
 *       YCoCg.to_RGB (:449), += 128 (:454), clip/astype(uint8) (:466)
 *
 * Conventions
 *   - Plain C, no C++ or torch types.  Every function returns VCF_OK (0) or a
 *     negative status; vcf_last_error() describes the last failure of the
 *     calling thread.
 *   - Buffers are caller-owned.  Pointers named *_dev are device (HBM)
 *     pointers, e.g. from vcf_malloc; the library never frees caller memory
 *     and keeps no reference after a call returns.
 *   - Frames are stored back to back.  An RGB frame is H x W x 3 uint8
 *     (row-major, channels interleaved, exactly the ndarray the reference's
 *     encode_read_fn returns).  A coefficient frame is Hp x Wp x 3 uint8 with
 *     Hp, Wp = H, W rounded up to the block size (vcf_dct_padded_shape): the
 *     array the reference hands to its entropy codec (2D-DCT.py:364).
 *   - Work is enqueued on `stream` (a hipStream_t, NULL = default stream)
 *     and is asynchronous; synchronise with vcf_stream_sync.
 */
#ifndef VCF_AMD_H
#define VCF_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VCF_OK 0
#define VCF_ERR_INVALID (-1)     /* bad argument (reference: ValueError)   */
#define VCF_ERR_HIP (-2)         /* HIP runtime failure                    */
#define VCF_ERR_UNSUPPORTED (-3) /* option not implemented on this path    */
#define VCF_ERR_TIMEOUT (-4)     /* a cross-rank exchange did not finish in time
                                    (the communicator is aborted)          */

/* element types of the stand-alone quantizer */
#define VCF_DTYPE_F32 0
#define VCF_DTYPE_F64 1
#define VCF_DTYPE_I16 2
#define VCF_DTYPE_I32 3
#define VCF_DTYPE_U8 4
#define VCF_DTYPE_U16 5

/* flags of the DCT path */
#define VCF_DCT_NO_SUBBANDS 1u   /* -x, --disable_subbands  (2D-DCT.py:40)  */
#define VCF_DCT_PERCEPTUAL 2u    /* -p, --perceptual_quantization (:38)    */

/* ---- runtime ----------------------------------------------------------- */
const char *vcf_last_error(void);
int vcf_version(int *major, int *minor);
int vcf_device_count(int *n);
int vcf_set_device(int device);
int vcf_get_device(int *device);
int vcf_device_sync(void);
int vcf_malloc(void **ptr_dev, size_t bytes);
int vcf_free(void *ptr_dev);
int vcf_host_alloc(void **ptr_host, size_t bytes); /* pinned */
int vcf_host_free(void *ptr_host);
int vcf_memcpy_htod(void *dst_dev, const void *src_host, size_t bytes, void *stream);
int vcf_memcpy_dtoh(void *dst_host, const void *src_dev, size_t bytes, void *stream);
int vcf_memcpy_dtod(void *dst_dev, const void *src_dev, size_t bytes, void *stream);
int vcf_memset(void *dst_dev, int value, size_t bytes, void *stream);
int vcf_stream_create(void **stream);
int vcf_stream_destroy(void *stream);
int vcf_stream_sync(void *stream);
int vcf_event_create(void **event);
int vcf_event_destroy(void *event);
int vcf_event_record(void *event, void *stream);
int vcf_event_sync(void *event);
/* n_pieces device copies in one launch: piece p moves table_dev[3p + 2] bytes
 * from src_dev + table_dev[3p] to dst_dev + table_dev[3p + 1] (int64 table in
 * device memory); e.g. per-frame code-streams packed for the gather */
int vcf_copy_pieces(const uint8_t *src_dev, const int64_t *table_dev, int64_t n_pieces, uint8_t *dst_dev,
                    void *stream);
/* later work on `stream` waits for `event` (hipStreamWaitEvent) */
int vcf_stream_wait_event(void *stream, void *event);
int vcf_event_elapsed_ms(void *start, void *stop, float *ms);

/* ---- DCT + deadzone path (2D-DCT.py, deadzone.py, YCoCg.py) ---------------- */

/* Hp, Wp for an H x W frame: 2D-DCT.py:208-209. */
int vcf_dct_padded_shape(int32_t H, int32_t W, int32_t block_size, int32_t *Hp, int32_t *Wp);

/* n_frames RGB frames (H x W x 3 u8 each) -> n_frames coefficient frames
 * (Hp x Wp x 3 u8 each, k + 128 modulo 256, subband layout unless
 * VCF_DCT_NO_SUBBANDS).  block_size is the -B option (2D-DCT.py:29): 8 runs
 * the fused 8x8 kernels, the other supported sizes (vcf_dct_block_size_supported)
 * the generic-B kernels; VCF_DCT_PERCEPTUAL takes any supported B (B != 8
 * through vcf_dct_perceptual_tables' resized tables).  Q >= 1 is the
 * deadzone quantization step (-q). */
int vcf_dct_dz_encode(const uint8_t *rgb_dev, int64_t n_frames, int32_t H, int32_t W,
                      int32_t block_size, int32_t Q, uint32_t flags, uint8_t *k_dev,
                      void *stream);



/* Inverse: n_frames coefficient frames (Hp x Wp x 3) -> RGB frames (H x W x 3),
 * the padding removed.  1 <= Q <= 32767 (the dequantizer works in int16). */
int vcf_dct_dz_decode(const uint8_t *k_dev, int64_t n_frames, int32_t H, int32_t W,
                      int32_t block_size, int32_t Q, uint32_t flags, uint8_t *rgb_dev,
                      void *stream);

/* 1 if block_size has a HIP transform: every 1 <= B <= 4096 -- compiled
 * kernels for the 38 5-smooth B <= 128 (every -L candidate 2, 4, ..., 128,
 * 2D-DCT.py:536), run-time-length kernels for the rest: rfftp plans with the
 * generic radfg/radbg passes, and the lengths pocketfft_r plans with
 * Bluestein (191, 199, 211, ...: fftblue over cfftp).  0 for B > 4096. */
int vcf_dct_block_size_supported(int32_t block_size);

/* -p's quantization tables for block size B (host only): the JPEG luma /
 * chroma tables of 2D-DCT.py:66-84 resized to B x B as :85-90 does
 * (cv2.resize, INTER_AREA for B < 8, INTER_LINEAR otherwise), B*B bytes each.
 * cv2 is not installed here: OpenCV's scalar resize code paths are restated,
 * unpinned by any reference output (parity unpinned for -p with B != 8). */
int vcf_dct_perceptual_tables(int32_t block_size, uint8_t *y_qss, uint8_t *c_qss);

/* The generic-B kernels for any supported block size, B = 8 included (tests
 * and A/B checks against the fused 8x8 kernels); same contract as
 * vcf_dct_dz_encode / vcf_dct_dz_decode. */
int vcf_dct_dz_encode_any(const uint8_t *rgb_dev, int64_t n_frames, int32_t H, int32_t W, int32_t block_size,
                          int32_t Q, uint32_t flags, uint8_t *k_dev, void *stream);
int vcf_dct_dz_decode_any(const uint8_t *k_dev, int64_t n_frames, int32_t H, int32_t W, int32_t block_size,
                          int32_t Q, uint32_t flags, uint8_t *rgb_dev, void *stream);

/* The -L rate-distortion search's own analysis/synthesis
 * (2D-DCT.py optimize_block_size :533-579), which differs from
 * encode_fn/decode_fn in its integer types and offset.  The search runs from
 * CoDec.__init__ (:99-103) before the deadzone offset 128 is assigned
 * (:106-109), so its self.offset is YCoCg's [0, 0, 0] (YCoCg.py:28-29):
 *   encode_k32: astype(float32) (no -128), from_RGB, analyze, get_subbands,
 *     quantize (:536-545) -> the int32 k array (Hp x Wp x 3 int32);
 *   decode_k32: Q*k in int32 (:561), get_blocks, the IDCT stored into int32,
 *     to_RGB in int32 (no +128), clip, uint8 (:562-568).
 * No VCF_DCT_PERCEPTUAL (the reference refuses -L with -p, :100-105). */
int vcf_dct_dz_encode_k32(const uint8_t *rgb_dev, int64_t n_frames, int32_t H, int32_t W, int32_t block_size,
                          int32_t Q, uint32_t flags, int32_t *k_dev, void *stream);
int vcf_dct_dz_decode_k32(const int32_t *k_dev, int64_t n_frames, int32_t H, int32_t W, int32_t block_size,
                          int32_t Q, uint32_t flags, uint8_t *rgb_dev, void *stream);

/* encode_fn / decode_fn with a quantizer other than deadzone (-a LloydMax):
 * 2D-DCT.py:106-109 sets self.offset = 0, so there is no -128 before the
 * colour transform and no +128 on the pixels; the quantizer sees the float32
 * coefficients (subband layout unless -x, -p weights applied, :313-340) and
 * hands back int16 coefficients (:399-410).  Replaces the same spans as
 * vcf_dct_dz_encode/decode minus the deadzone quantizer; any supported B. */
int vcf_dct_raw_encode(const uint8_t *rgb_dev, int64_t n_frames, int32_t H, int32_t W, int32_t block_size,
                       uint32_t flags, float *coef_dev, void *stream);
int vcf_dct_raw_decode(const int16_t *coef_dev, int64_t n_frames, int32_t H, int32_t W, int32_t block_size,
                       uint32_t flags, uint8_t *rgb_dev, void *stream);



/* ---- 2D-DWT + deadzone path (2D-DWT.py, deadzone.py, YCoCg.py) ---------------- */

/* Index of a pywt wavelet name ("db5", "bior4.4", ... -- the -w option,
 * 2D-DWT.py:45) in the library's filter table. */
int vcf_wavelet_index(const char *name, int32_t *index);

/* Subband shapes (level l = 1..levels in sub_h[l-1], sub_w[l-1]; mode 'per'
 * halves with ceil), bytes of one frame's packed subbands, and the device
 * workspace one frame needs.  Any output pointer may be NULL. */
int vcf_dwt_layout(int32_t H, int32_t W, int32_t levels, int32_t *sub_h, int32_t *sub_w, int64_t *packed_bytes,
                   int64_t *workspace_bytes_per_frame);

/* n_frames RGB frames -> n_frames packed subband sets, each laid out in the
 * order 2D-DWT.py's write_decom_fn (:162-200) writes its files: LL_L
 * (uint16 little-endian, h_L x w_L x 3, k + 128 wrapped), then for r = L..1
 * LH_r, HL_r, HH_r (uint8, h_r x w_r x 3, k + 128 wrapped).  Replaces
 * 2D-DWT.py:57-78 up to the TIFF writer: astype(int16), from_RGB (:62),
 * pywt.wavedec2 mode 'per' per channel (:64), quantize_decom_fn (:67).
 * workspace_dev: n_frames * workspace_bytes_per_frame bytes. */
int vcf_dwt_dz_encode(const uint8_t *rgb_dev, int64_t n_frames, int32_t H, int32_t W, int32_t wavelet,
                      int32_t levels, int32_t Q, uint8_t *packed_dev, void *workspace_dev, void *stream);

/* Inverse: packed subbands -> RGB frames of 2*ceil(H/2) x 2*ceil(W/2) x 3
 * (what pywt.waverec2 returns; the reference writes that size too).
 * Replaces 2D-DWT.py:80-101 after the TIFF reader.  1 <= Q <= 32767.
 * Coarsest subbands shorter than filter_length/2 (pywt's short-input code
 * path) run on the separable kernels. */
int vcf_dwt_dz_decode(const uint8_t *packed_dev, int64_t n_frames, int32_t H, int32_t W, int32_t wavelet,
                      int32_t levels, int32_t Q, uint8_t *rgb_dev, void *workspace_dev, void *stream);

/* A/B switch of vcf_dwt_dz_decode, process-wide: on = 1 (default) runs the
 * inverse levels 2 and 1 in one launch where the planes halve evenly (LL1
 * stays on chip), 0 one launch per level.  Identical bytes either way. */
int vcf_dwt_set_inverse_band21(int32_t on);

/* Opt-in lifting form of the two calls above for bior4.4 (CDF 9/7) only
 * (VCF_ERR_INVALID for other wavelets): same arguments, buffers, layout and
 * workspace, four lifting steps per axis in place of pywt's convolution.
 * NOT bit-exact: every index and decoded byte lies within +-1 of
 * vcf_dwt_dz_encode / _decode's (measured, DESIGN.md §4.5, the lifting form).  No counterpart
 * in the reference -- an extension for callers who accept that tolerance. */
int vcf_dwt_dz_encode_lift(const uint8_t *rgb_dev, int64_t n_frames, int32_t H, int32_t W, int32_t wavelet,
                           int32_t levels, int32_t Q, uint8_t *packed_dev, void *workspace_dev, void *stream);
int vcf_dwt_dz_decode_lift(const uint8_t *packed_dev, int64_t n_frames, int32_t H, int32_t W, int32_t wavelet,
                           int32_t levels, int32_t Q, uint8_t *rgb_dev, void *workspace_dev, void *stream);
/* A/B switch of the lifting calls, process-wide: fused = 1 (default) runs
 * levels in pairs (1 + 2, 3 + 4 and their inverses) in one launch, 0 one
 * launch per level.  Both give identical bytes (tests/test_dwt_lift_gpu.py). */
int vcf_dwt_lift_set_fused(int32_t fused);
/* Diagnostic of the lifting form's precision (one frame, bior4.4): its float64
 * subband coefficients before quantization.  coef_dev receives, for levels
 * l = 1..levels, the details [LH, HL, HH][Y, Co, Cg][h_l x w_l] (the shapes of
 * vcf_dwt_layout), then LL_levels [Y, Co, Cg][h x w]; packed_dev (packed bytes
 * of vcf_dwt_layout) and workspace_dev are scratch. */
int vcf_dwt_lift_analyze_f64(const uint8_t *rgb_dev, int32_t H, int32_t W, int32_t levels, double *coef_dev,
                             uint8_t *packed_dev, void *workspace_dev, void *stream);



/* ---- IPP temporal tools (IPP_DCT.py) --------------------------------------------- */

/* Motion field of cur against ref (H x W x 3 u8 each): IPP.block_matching
 * (IPP_DCT.py:344-376) -- cv2 RGB2GRAY (A10), then per bs x bs block of the
 * full-block area the (dx, dy) of the full search (fast = 0,
 * _process_block_row :207-246) or the three-step search (fast = 1,
 * _three_step_search :159-204) over [-sr, sr].  mv_dev: (H/bs) x (W/bs) x 2
 * float32; gray_workspace_dev: 2*H*W bytes.  bs <= 64, sr <= 32. */
int vcf_ipp_block_match(const uint8_t *ref_rgb_dev, const uint8_t *cur_rgb_dev, int32_t H, int32_t W, int32_t bs,
                        int32_t sr, int32_t fast, float *mv_dev, uint8_t *gray_workspace_dev, void *stream);

/* Block-matching kernel choice (benchmarking and tests; process-wide):
 * 0 = the word kernels -- full search on 4-pixel words (v_alignbyte +
 * v_sad_u8, one lane per candidate) when bs % 4 == 0, and for bs = 16 the
 * three-step search in parallel rounds of its 8 neighbours; 1 = the byte
 * kernels (full search) and the serial three-step kernel.  Both give
 * identical motion fields. */
int vcf_ipp_set_full_search_variant(int32_t variant);

/* IPP.motion_compensate (IPP_DCT.py:378-395). */
int vcf_ipp_motion_compensate(const uint8_t *ref_rgb_dev, const float *mv_dev, int32_t H, int32_t W, int32_t bs,
                              uint8_t *out_rgb_dev, void *stream);

/* residual_shifted = clip(cur - comp + 128, 0, 255) (IPP_DCT.py:547-551). */
int vcf_ipp_residual(const uint8_t *cur_dev, const uint8_t *comp_dev, int64_t n, uint8_t *out_dev, void *stream);

/* recon = clip(comp + rec - 128, 0, 255) (IPP_DCT.py:559-561, 788-790). */
int vcf_ipp_reconstruct(const uint8_t *comp_dev, const uint8_t *rec_dev, int64_t n, uint8_t *out_dev, void *stream);

/* -R block-level RDO of IPP.temporal_filter (IPP_DCT.py:441-536): for every
 * full bs x bs block, IPP.rdo_block_decision (:290-342) on the cv2 RGB2GRAY
 * luma of cur and of its motion compensation comp -- float64 pocketfft DCT,
 * round(x / Q) to int16, float32 dequantization and IDCT, numpy-pairwise
 * mean squared error, get_rate (:265-288) -- and the mode with the smaller
 * D + lambda R (ties to inter).  modes_dev: (H/bs) x (W/bs) u8, 1 = I
 * (intra), 0 = P; costs_dev (NULL or 4 doubles per block): D_inter,
 * R_inter, D_intra, R_intra.  bs in {2, 4, 8, 12, 16, 24, 32}. */
int vcf_ipp_rdo_modes(const uint8_t *cur_dev, const uint8_t *comp_dev, int32_t H, int32_t W, int32_t bs, int32_t Q,
                      double lambda, uint8_t *modes_dev, double *costs_dev, void *stream);

/* The frame -R hands to the spatial codec (:489-505): P blocks
 * clip(cur - comp + 128), I blocks cur, pixels outside full blocks 128. */
int vcf_ipp_rdo_residual(const uint8_t *cur_dev, const uint8_t *comp_dev, const uint8_t *modes_dev, int32_t H,
                         int32_t W, int32_t bs, uint8_t *out_dev, void *stream);

/* Mode-aware reconstruction (:512-526, decoder :770-790): P blocks
 * clip(comp + rec - 128), I blocks rec, pixels outside full blocks 0. */
int vcf_ipp_rdo_reconstruct(const uint8_t *comp_dev, const uint8_t *rec_dev, const uint8_t *modes_dev, int32_t H,
                            int32_t W, int32_t bs, uint8_t *out_dev, void *stream);

/* ---- CBAAC entropy codec (CBAAC.py), host code --------------------------------- */

/* Worst-case code-stream bytes for n symbols. */
int64_t vcf_cbaac_bound(int64_t n_symbols);

/* Context-based adaptive arithmetic coding of n byte symbols with a model of
 * the previous `order` symbols (0..8): CBAAC.CoDec._encode (CBAAC.py:114-131)
 * with AdaptiveModel/ContextManager (:17-69) exactly and the A8 coder.  Host
 * pointers.  Writes the big-endian bit stream (zero padded) the reference
 * appends after its header (:81-95); *out_bytes / *out_bits receive its
 * length. */
int vcf_cbaac_encode(const uint8_t *symbols, int64_t n, int32_t order, uint8_t *out, int64_t out_capacity,
                     int64_t *out_bytes, int64_t *out_bits);

/* Inverse (CBAAC.py:133-150): n symbols from nbytes of code-stream. */
int vcf_cbaac_decode(const uint8_t *bytes, int64_t nbytes, int64_t n, int32_t order, uint8_t *symbols_out);

/* The model alone: the (low, high, total) triple given to the coder for each
 * symbol (3*n int32), for parity checks against the reference's model. */
int vcf_cbaac_model_trace(const uint8_t *symbols, int64_t n, int32_t order, int32_t *triples);

/* ---- tiled CBAAC on the GPU ------------------------------
 * The flattened symbols split into consecutive segments of seg_len symbols
 * (a multiple of 256); each segment is coded exactly as vcf_cbaac_encode
 * codes it alone: CBAAC.CoDec._encode (CBAAC.py:114-131) with a fresh
 * ContextManager (:49-69) and history per segment, one wave per segment.
 * Orders 0 and 1 (VCF_ERR_UNSUPPORTED above).  Device pointers; the
 * container (segment sizes + payload) is vcf_amd/tcbaac.py's. */
int64_t vcf_cbaac_tiled_segments(int64_t n, int64_t seg_len);
/* scratch bytes (ws_dev) for vcf_cbaac_tiled_encode / _trace */
int64_t vcf_cbaac_tiled_workspace(int64_t n, int64_t seg_len);
/* an out_capacity that always suffices */
int64_t vcf_cbaac_tiled_bound(int64_t n, int64_t seg_len);
/* Segments packed back to back into out_dev; seg_bytes_dev (segments + 1
 * int64) receives each segment's byte count and, last, the total (> capacity
 * means the output was cut: retry with vcf_cbaac_tiled_bound bytes). */
int vcf_cbaac_tiled_encode(const uint8_t *sym_dev, int64_t n, int32_t order, int64_t seg_len, uint8_t *out_dev,
                           int64_t out_capacity, int64_t *seg_bytes_dev, void *ws_dev, void *stream);
/* Kernel choice (process-wide; A/B and tests): 0 = automatic -- order 0 codes
 * one segment per LANE (64 segments per wave, each with its own model in
 * LDS) once a call has at least 4608 segments to encode / 6144 to decode
 * (all frames of the call), else one segment per wave
 * (64 lanes share one model: a shorter time per segment); 1 = one segment per
 * wave always; 2 = one segment per lane for order 0 always.  Same bytes. */
int vcf_cbaac_tiled_set_variant(int32_t variant);
/* The model alone: the (low, high, total) triple handed to the coder for
 * every symbol (3*n int32), segment by segment (parity checks). */
int vcf_cbaac_tiled_trace(const uint8_t *sym_dev, int64_t n, int32_t order, int64_t seg_len, int32_t *triples_dev,
                          int64_t *seg_bytes_dev, void *ws_dev, void *stream);
/* Inverse: segment s's bytes are in_dev[offs[s] .. offs[s+1]) (segments + 1
 * int64 byte offsets, device); n symbols out. */
int vcf_cbaac_tiled_decode(const uint8_t *in_dev, const int64_t *seg_offsets_dev, int64_t n, int32_t order,
                           int64_t seg_len, uint8_t *sym_dev, void *stream);
/* Prior-seeded segments, orders 0 and 1 (container version 2; not in the
 * reference, which starts every model from 256 ones): the frame's order-0
 * prior f[s] = 1 + floor(hist[s] * 8192 / n) (256 uint16 in prior_dev,
 * 8-byte aligned; hist_dev = 256 uint32 of scratch) seeds every model of
 * every segment (order 1: all 256 contexts), which then adapts by
 * CBAAC.py:32-36.  Each segment's bytes equal vcf_cbaac_encode_prior of that
 * segment alone. */
int vcf_cbaac_tiled_prior(const uint8_t *sym_dev, int64_t n, uint16_t *prior_dev, uint32_t *hist_dev, void *stream);
int vcf_cbaac_tiled_encode_prior(const uint8_t *sym_dev, int64_t n, int32_t order, const uint16_t *prior_dev,
                                 int64_t seg_len, uint8_t *out_dev, int64_t out_capacity, int64_t *seg_bytes_dev,
                                 void *ws_dev, void *stream);
int vcf_cbaac_tiled_decode_prior(const uint8_t *in_dev, const int64_t *seg_offsets_dev, int64_t n, int32_t order,
                                 const uint16_t *prior_dev, int64_t seg_len, uint8_t *sym_dev, void *stream);
/* Batches of frames, each coded exactly as the single-frame calls code it,
 * in one launch per stage (a frame's segments alone fill few waves): n_frames
 * (<= 65535) frames of frame_symbols symbols, frame f's symbols at sym_dev +
 * f * frame_stride (any alignment); priors_dev = n_frames x 256 uint16 (frame
 * f's prior at priors_dev + 256 f; NULL = fresh models, container version 1),
 * hist_dev = n_frames x 256 uint32 of scratch; frame f's packed segments at
 * out_dev + f * out_frame_capacity, its segment byte counts and total at
 * seg_bytes_dev + f * (segments + 1); ws_dev = vcf_cbaac_tiled_frames_workspace
 * bytes.  Decode: frame f's segment offsets at seg_offsets_dev + f * (segments
 * + 1), offsets into in_dev; its symbols to sym_dev + f * out_frame_stride. */
int64_t vcf_cbaac_tiled_frames_workspace(int64_t n_frames, int64_t frame_symbols, int64_t seg_len);
int vcf_cbaac_tiled_prior_frames(const uint8_t *sym_dev, int64_t n_frames, int64_t frame_symbols,
                                 int64_t frame_stride, uint16_t *priors_dev, uint32_t *hist_dev, void *stream);
int vcf_cbaac_tiled_encode_frames(const uint8_t *sym_dev, int64_t n_frames, int64_t frame_symbols,
                                  int64_t frame_stride, int32_t order, const uint16_t *priors_dev, int64_t seg_len,
                                  uint8_t *out_dev, int64_t out_frame_capacity, int64_t *seg_bytes_dev, void *ws_dev,
                                  void *stream);
int vcf_cbaac_tiled_decode_frames(const uint8_t *in_dev, const int64_t *seg_offsets_dev, int64_t n_frames,
                                  int64_t frame_symbols, int32_t order, const uint16_t *priors_dev, int64_t seg_len,
                                  uint8_t *sym_dev, int64_t out_frame_stride, void *stream);
/* Prior classes (container version 3; not in the reference): nclass
 * (1 .. 256) prior rows per frame instead of one.  Segment s of a frame's
 * `segments` takes row floor(s * nclass / segments) -- consecutive runs of
 * segments share a row, so for DCT indices in the subband layout and nclass =
 * 8 a row is (about) one subband row i, whose statistics differ the most --
 * and row c = 1 + floor(hist_c[s] * 8192 / n_c) over the symbols of class c's
 * segments (nclass = 1: the version-2 prior).  priors_dev = n_frames x nclass
 * x 256 uint16 (frame f, class c at + 256 (f nclass + c); 8-byte aligned),
 * hist_dev = as many uint32 of scratch; the rest as the _frames calls.  Each
 * segment's bytes equal vcf_cbaac_encode_prior of that segment alone with
 * its class's row. */
int vcf_cbaac_tiled_prior_classes(const uint8_t *sym_dev, int64_t n_frames, int64_t frame_symbols,
                                  int64_t frame_stride, int64_t seg_len, int32_t nclass, uint16_t *priors_dev,
                                  uint32_t *hist_dev, void *stream);
int vcf_cbaac_tiled_encode_classes(const uint8_t *sym_dev, int64_t n_frames, int64_t frame_symbols,
                                   int64_t frame_stride, int32_t order, const uint16_t *priors_dev, int32_t nclass,
                                   int64_t seg_len, uint8_t *out_dev, int64_t out_frame_capacity,
                                   int64_t *seg_bytes_dev, void *ws_dev, void *stream);
int vcf_cbaac_tiled_decode_classes(const uint8_t *in_dev, const int64_t *seg_offsets_dev, int64_t n_frames,
                                   int64_t frame_symbols, int32_t order, const uint16_t *priors_dev, int32_t nclass,
                                   int64_t seg_len, uint8_t *sym_dev, int64_t out_frame_stride, void *stream);
/* host: version 3's container pieces for a batch of frames -- the segment
 * sizes of each row as unsigned LEB128 varints (row r's bytes end at
 * out[row_end[r]]), and each frame's nclass prior rows stored sparsely
 * (uint32 nclass; per row uint16 m, the m symbols with a frequency != 1, their
 * m uint16 frequencies; frame f's bytes end at out[frame_end[f]]). */
int vcf_leb128_encode_rows(const int64_t *v, int64_t rows, int64_t cols, uint8_t *out, int64_t capacity,
                           int64_t *row_end);
int vcf_prior_rows_sparse(const uint16_t *priors, int64_t frames, int32_t nclass, uint8_t *out, int64_t capacity,
                          int64_t *frame_end);
/* host, orders 0 / 1: vcf_cbaac_encode / _decode with every model seeded by prior (256 uint16, each >= 1) */
int vcf_cbaac_encode_prior(const uint8_t *symbols, int64_t n, int32_t order, const uint16_t *prior, uint8_t *out,
                           int64_t out_capacity, int64_t *out_bytes, int64_t *out_bits);
int vcf_cbaac_decode_prior(const uint8_t *bytes, int64_t nbytes, int64_t n, int32_t order, const uint16_t *prior,
                           uint8_t *symbols_out);

/* ---- CBAHC entropy codec (CBAHC.py), host code --------------------------------- */

/* Worst-case code-stream bytes for n symbols. */
int64_t vcf_cbahc_bound(int64_t n_symbols);

/* Context-based adaptive Huffman coding of n byte symbols (order 0..7):
 * CBAHC.CoDec.compress_fn (CBAHC.py:169-221) bit for bit -- per symbol a
 * Huffman tree from the context's counts (:38-78), its code (:81-106), then
 * the count update.  Big-endian bits, zero padded; *out_bits = exact count
 * (the reference keeps it in its side file). */
int vcf_cbahc_encode(const uint8_t *symbols, int64_t n, int32_t order, uint8_t *out, int64_t out_capacity,
                     int64_t *out_bytes, int64_t *out_bits);

/* Inverse (CBAHC.py:226-276): n symbols from the first nbits bits. */
int vcf_cbahc_decode(const uint8_t *bytes, int64_t nbits, int64_t n, int32_t order, uint8_t *symbols_out);

/* ---- frame ingest: PNG reader (host code) ------------------------------------ */

/* Size of a PNG in memory and whether vcf_png_decode_rgb covers it (bit
 * depth 8, colour type 0/2/3/4/6, not interlaced). */
int vcf_png_info(const uint8_t *data, int64_t nbytes, int32_t *H, int32_t *W, int32_t *supported);

/* PNG bytes -> H x W x 3 RGB u8 (host buffer of out_capacity bytes): what
 * EIC.encode_read_fn reads (entropy_image_coding.py:51-65; A9: PIL's
 * convert("RGB") -- gray replicated, alpha dropped, palette looked up).
 * VCF_ERR_UNSUPPORTED for PNGs outside vcf_png_info's set (the caller falls
 * back to another reader), VCF_ERR_INVALID for corrupt files. */
int vcf_png_decode_rgb(const uint8_t *data, int64_t nbytes, uint8_t *rgb_out, int64_t out_capacity);

/* RGB u8 (H x W x 3, host) -> PNG file bytes: 8-bit truecolour, Up-filtered
 * scanlines, one zlib stream at `level` deflated in 1 MiB pieces on up to
 * `threads` threads (pigz's construction: each piece primed with the previous
 * 32 KiB, sync-flushed, adler32 combined).  The writer of the decode side's
 * PNGs (EIC.decode_write_fn, entropy_image_coding.py:101-112) and of IPP's
 * frame dumps: pixel-exact, not byte-identical to other PNG writers.
 * out_capacity >= vcf_png_encode_bound(H, W) always suffices; *out_bytes
 * receives the file size. */
int vcf_png_encode_rgb(const uint8_t *rgb, int32_t H, int32_t W, int32_t level, int32_t threads, uint8_t *out,
                       int64_t out_capacity, int64_t *out_bytes);
int64_t vcf_png_encode_bound(int32_t H, int32_t W);

/* ---- TIFF strip deflate on the GPU (TIFF.py:23-31, the default -c) ----------
 * zlib.compress(strip, level) for every strip of a batch of frames, byte for
 * byte (zlib 1.2.11 deflate_slow, windowBits 15, memLevel 8): what
 * tifffile.imwrite(..., compression='zlib') stores per RowsPerStrip strip
 * (TIFF.py:29; host path vcf_amd/codec/tiff.py _deflate_strips).  Frame f is
 * in_dev[f*frame_bytes, (f+1)*frame_bytes), cut into strips of strip_bytes
 * (the last one shorter); strip s = f*spf + k, spf = vcf_zlib_strip_count,
 * is written to out_dev + s*slot_bytes and its length to sizes_dev[s]
 * (-1: slot too small).  level 4..9 (VCF_ERR_UNSUPPORTED otherwise);
 * strip_bytes <= 65536 (tifffile's strips for rows up to 64 KB);
 * slot_bytes a multiple of 4 >= vcf_zlib_bound(strip_bytes); ws_dev holds
 * vcf_zlib_workspace(total strips) bytes (16-byte aligned; out_dev and
 * sizes_dev 4-byte aligned) -- ~1.15 MB per strip, at most the workspace
 * budget whatever the batch: past that the strips are coded in rounds that
 * reuse it.  The budget is fixed per device on first use: a quarter of the
 * memory free then, clamped to 3.9..40 GB; vcf_zlib_set_workspace_budget(b)
 * sets it for the current device (0 restores the default; b at least one
 * strip's workspace), after which vcf_zlib_workspace must be asked again.  The call is asynchronous on `stream`;
 * internally part of each round runs on library streams forked from and
 * joined back to it, so the caller sees ordinary stream semantics. */
int64_t vcf_zlib_bound(int64_t strip_bytes);
int64_t vcf_zlib_workspace(int64_t n_strips);
int vcf_zlib_set_workspace_budget(int64_t bytes);
/* the largest strip_bytes vcf_zlib_strips takes (65536: frames with rows of
 * more than 64 KB -- 1-row strips past 21845 RGB pixels -- stay on the host writer) */
int32_t vcf_zlib_max_strip(void);
int64_t vcf_zlib_strip_count(int64_t frame_bytes, int32_t strip_bytes);
int vcf_zlib_strips(const uint8_t *in_dev, int64_t n_frames, int64_t frame_bytes, int32_t strip_bytes, int32_t level,
                    uint8_t *out_dev, int64_t slot_bytes, int32_t *sizes_dev, void *ws_dev, void *stream);

/* ---- TIFF strip inflate on the GPU (TIFF.py:33-39, the decode side of -c TIFF)
 * zlib.decompress for every strip of a batch: strip s is comp_len_dev[s] bytes
 * of a zlib stream at comp_dev + comp_off_dev[s], inflated to
 * out_dev + out_off_dev[s], which must come to exactly out_len_dev[s] bytes
 * (the TIFF's rows per strip x row bytes).  status_dev[s] = 0, or < 0 when the
 * stream is not one zlib accepts with that length (-1 header, -2 block, -3
 * code, -4 distance, -5 length, -6 adler32, -7 input overrun, -8 an
 * over-subscribed or incomplete code-length set, -9 no end-of-block code,
 * -10 a negative length: nothing read or written).  Device arrays, which the
 * kernel trusts: offsets and lengths must lie inside comp_dev and out_dev
 * (vcf_amd/zlib_gpu.py checks them on the host first); RFC 1950/1951,
 * stored, fixed and dynamic blocks. */
int vcf_inflate_strips(const uint8_t *comp_dev, const int64_t *comp_off_dev, const int32_t *comp_len_dev,
                       int64_t n_strips, uint8_t *out_dev, const int64_t *out_off_dev, const int32_t *out_len_dev,
                       int32_t *status_dev, void *stream);

/* ---- deadzone quantizer plug-in (deadzone.py:95-117, assumption A5) ---------- */

/* k[i] = (int32)(x[i] / Q), truncation toward zero; the division is float32
 * for VCF_DTYPE_F32 input and float64 for every other input type (numpy true
 * division).  Replaces deadzone.CoDec.quantize_fn (deadzone.py:95-102). */
int vcf_deadzone_quantize(const void *x_dev, int32_t x_dtype, int64_t n, int32_t Q, int32_t *k_dev,
                          void *stream);

/* y[i] = Q * k[i] in k's type (VCF_DTYPE_I16 or VCF_DTYPE_I32), wrapping.
 * Replaces deadzone.CoDec.dequantize_fn (deadzone.py:107-117). */
int vcf_deadzone_dequantize(const void *k_dev, int32_t k_dtype, int64_t n, int32_t Q, void *y_dev,
                            void *stream);

/* ---- §8(f) row 4: the YCrCb and LloydMax plug-ins ------------------------------
 * YCrCb (src/YCrCb.py:25-72): the stand-alone pixel codec.  Its transform,
 * color_transforms.YCrCb, is not vendored: OpenCV's integer RGB<->YCrCb on
 * uint8 is assumed (A12; parity unpinned).  n_px pixels of 3 interleaved
 * channels.  Note: 2D-DCT.py / 2D-DWT.py with -t YCrCb still convert with
 * YCoCg (they bind from_RGB/to_RGB from color_transforms.YCoCg, 2D-DCT.py:22-23,
 * 2D-DWT.py:19-20), so they use the YCoCg entry points above. */
int vcf_ycrcb_from_rgb(const uint8_t *rgb_dev, int64_t n_px, uint8_t *ycrcb_dev, void *stream);
int vcf_ycrcb_to_rgb(const uint8_t *ycrcb_dev, int64_t n_px, uint8_t *rgb_dev, void *stream);
/* YCrCb.encode (:33-51) with -a deadzone: from_RGB, int16, (x / Q) truncated, uint16. */
int vcf_ycrcb_dz_encode(const uint8_t *rgb_dev, int64_t n_px, int32_t Q, uint16_t *k_dev, void *stream);
/* YCrCb.decode (:53-72): Q * k in uint16, int16, uint8, to_RGB, clip. */
int vcf_ycrcb_dz_decode(const uint16_t *k_dev, int64_t n_px, int32_t Q, uint8_t *rgb_dev, void *stream);

/* ---- the stand-alone pixel codecs YCoCg.py and deadzone.py -------------------
 * YCoCg.encode (src/YCoCg.py:33-56) with -a deadzone: img.astype(int16),
 * from_RGB into int16 (A4, truncated toward zero), += offset 0 (:27-28),
 * deadzone (x / Q) truncated (A5), astype(uint16).  n_px pixels of 3
 * interleaved channels; k_dev n_px * 3 uint16. */
int vcf_ycocg_dz_encode(const uint8_t *rgb_dev, int64_t n_px, int32_t Q, uint16_t *k_dev, void *stream);
/* YCoCg.decode (:58-85): astype(int16), Q * k in int16 (1 <= Q <= 32767, else
 * VCF_ERR_UNSUPPORTED), to_RGB in int16 (A4, wrapping), clip(0, 255), uint8. */
int vcf_ycocg_dz_decode(const uint16_t *k_dev, int64_t n_px, int32_t Q, uint8_t *rgb_dev, void *stream);
/* YCoCg.py with -a LloydMax (:29-30, offset [-128, 0, 0]): the int16 YCoCg
 * image (A4) with offset0 added to Y, for the LloydMax entry points below; and
 * back: Y - offset0, to_RGB in int16, clip(0, 255), uint8. */
int vcf_ycocg_i16_from_rgb(const uint8_t *rgb_dev, int64_t n_px, int32_t offset0, int16_t *out_dev, void *stream);
int vcf_ycocg_i16_to_rgb(const int16_t *in_dev, int64_t n_px, int32_t offset0, uint8_t *rgb_dev, void *stream);
/* deadzone.encode (src/deadzone.py:67-79): astype(int16), (x / Q) truncated,
 * astype(uint8), elementwise over n bytes. */
int vcf_dz_u8_encode(const uint8_t *x_dev, int64_t n, int32_t Q, uint8_t *k_dev, void *stream);
/* deadzone.decode (:81-93): Q * k in uint8 (wrapping; 1 <= Q <= 255, the
 * Python-int-times-uint8 result type, else VCF_ERR_UNSUPPORTED). */
int vcf_dz_u8_decode(const uint8_t *k_dev, int64_t n, int32_t Q, uint8_t *y_dev, void *stream);

/* LloydMax (src/LloydMax.py:75-143).  Per channel c of an n_px x channels
 * array: counts = numpy.histogram(x[..., c], bins=max-min+1, range=(min, max))
 * (numpy 1.26's arithmetic; int64 counts, channel-major, zeroed here), the
 * glue's +1, the Lloyd-Max design of scalar_quantization's LloydMax_Quantizer
 * (un-vendored; A13, unpinned: the textbook design, oracle/plugins.py),
 * k = searchsorted(thresholds, x, 'right') stored with a C cast into k's type,
 * y = centroids[k] truncated into y's integer type.  dtypes: VCF_DTYPE_U8,
 * I16, U16, F32 (histogram/encode input, encode output).  vcf_lm_levels returns
 * the number of levels N = ceil((max - min + 1) / Q) or an error (< 0). */
int vcf_lm_levels(int32_t Q_step, int32_t min_val, int32_t max_val);
int vcf_lm_histogram(const void *x_dev, int32_t x_dtype, int64_t n_px, int32_t channels, int32_t min_val,
                     int32_t max_val, int64_t *counts_dev, void *stream);
/* Host memory: counts (n_bins, already +1) -> centroids (N doubles); returns N or an error. */
int vcf_lm_design(const int64_t *counts, int32_t n_bins, int32_t Q_step, int32_t min_val, double *centroids);
/* centroids_dev: channels x n_levels doubles (channel-major). */
int vcf_lm_encode(const void *x_dev, int32_t x_dtype, int64_t n_px, int32_t channels, const double *centroids_dev,
                  int32_t n_levels, void *k_dev, int32_t k_dtype, void *stream);
/* *bad_dev is set to 1 when an index is outside [-N, N) (numpy's IndexError); the caller zeroes it. */
int vcf_lm_decode(const void *k_dev, int32_t k_dtype, int64_t n_px, int32_t channels, const double *centroids_dev,
                  int32_t n_levels, void *y_dev, int32_t y_dtype, int32_t *bad_dev, void *stream);

/* ---- cross-rank exchange on RCCL over xGMI -------------------
 * Frames shard across one process per GPU with no collective on the data
 * path; the one exchange step of the III / IPP drivers is after coding: an
 * all-gather of the per-frame code-stream sizes and a gather of the
 * variable-length payloads to rank 0.  It replaces the point where the
 * reference's sequential frame loop has every coded frame in one process
 * (src/III.py:77-115 encode, :132-144 decode).  librccl is opened on first
 * use (dlopen); without it these return VCF_ERR_UNSUPPORTED.  Buffers are
 * device pointers, work is enqueued on `stream`. */
#define VCF_COMM_ID_BYTES 128
#define VCF_COMM_SUM 0
#define VCF_COMM_MAX 1
#define VCF_COMM_MIN 2
typedef struct vcf_comm *vcf_comm_t;

/* One rank creates the id (ncclGetUniqueId) and hands it to the others
 * out of band (vcf_amd/comm.py: a TCP host group). */
int vcf_comm_unique_id(uint8_t *id, size_t capacity);
/* Collective over `world` processes, each with its device already set
 * (vcf_set_device).  The communicator is non-blocking (ncclConfig_t
 * blocking = 0): initialisation and every enqueue below are polled against
 * a deadline of timeout_ms (<= 0: VCF_COMM_TIMEOUT_MS from the environment,
 * else 120000); past it the communicator is aborted (ncclCommAbort) and the
 * call returns VCF_ERR_TIMEOUT instead of hanging.  vcf_comm_init =
 * vcf_comm_init_timeout(..., 0). */
int vcf_comm_init(vcf_comm_t *comm, const uint8_t *id, int rank, int world);
int vcf_comm_init_timeout(vcf_comm_t *comm, const uint8_t *id, int rank, int world, int64_t timeout_ms);
/* Wait until everything enqueued on `stream` has finished, within the
 * communicator's timeout; past it (or on an asynchronous RCCL error) the
 * communicator is aborted and VCF_ERR_TIMEOUT (VCF_ERR_HIP) returned. */
int vcf_comm_wait(vcf_comm_t comm, void *stream);
int vcf_comm_destroy(vcf_comm_t comm);
int vcf_comm_rank(vcf_comm_t comm, int *rank, int *world);
/* recv_dev[r * count + i] = rank r's send_dev[i] (ncclAllGather, int64). */
int vcf_comm_allgather_i64(vcf_comm_t comm, const int64_t *send_dev, int64_t count, int64_t *recv_dev,
                           void *stream);
/* Element-wise VCF_COMM_SUM / MAX / MIN over ranks (ncclAllReduce, float64). */
int vcf_comm_allreduce_f64(vcf_comm_t comm, const double *send_dev, double *recv_dev, int64_t count, int op,
                           void *stream);
/* Gather with per-rank byte counts: rank r sends counts[r] bytes (= send_bytes)
 * and the root receives them packed in rank order in recv_dev.  counts (host,
 * `world` entries, the same on every rank -- e.g. from the size all-gather).
 * One grouped ncclSend per peer, P-1 concurrent ncclRecv on the root: each
 * xGMI peer uses its own link to the root (RCCL has no gatherv). */
int vcf_comm_gatherv(vcf_comm_t comm, const void *send_dev, int64_t send_bytes, void *recv_dev,
                     const int64_t *counts, int root, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* VCF_AMD_H */
