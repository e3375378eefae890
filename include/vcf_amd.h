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

/* element types of the stand-alone quantizer */
#define VCF_DTYPE_F32 0
#define VCF_DTYPE_F64 1
#define VCF_DTYPE_I16 2
#define VCF_DTYPE_I32 3
#define VCF_DTYPE_U8 4

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
int vcf_event_elapsed_ms(void *start, void *stop, float *ms);

/* ---- DCT + deadzone path (2D-DCT.py, deadzone.py, YCoCg.py) ---------------- */

/* Hp, Wp for an H x W frame: 2D-DCT.py:208-209. */
int vcf_dct_padded_shape(int32_t H, int32_t W, int32_t block_size, int32_t *Hp, int32_t *Wp);

/* n_frames RGB frames (H x W x 3 u8 each) -> n_frames coefficient frames
 * (Hp x Wp x 3 u8 each, k + 128 modulo 256, subband layout unless
 * VCF_DCT_NO_SUBBANDS).  block_size must be 8 (the -B default); Q >= 1 is the
 * deadzone quantization step (-q). */
int vcf_dct_dz_encode(const uint8_t *rgb_dev, int64_t n_frames, int32_t H, int32_t W,
                      int32_t block_size, int32_t Q, uint32_t flags, uint8_t *k_dev,
                      void *stream);

/* Same as vcf_dct_dz_encode with an explicit kernel choice (benchmarking and
 * tests): 0 = automatic, 1 = lane-per-block tile kernel (the default),
 * 2 = diagnostic: variant 1's arithmetic with no memory traffic (writes one
 * word per block, not the coefficients; power-of-two Q only),
 * 3 = column-per-lane tile kernel (8 lanes per block, LDS transpose).
 * Variants 1 and 3 produce identical bytes. */
int vcf_dct_dz_encode_variant(int variant, const uint8_t *rgb_dev, int64_t n_frames, int32_t H,
                              int32_t W, int32_t block_size, int32_t Q, uint32_t flags,
                              uint8_t *k_dev, void *stream);

/* Inverse: n_frames coefficient frames (Hp x Wp x 3) -> RGB frames (H x W x 3),
 * the padding removed.  1 <= Q <= 32767 (the dequantizer works in int16). */
int vcf_dct_dz_decode(const uint8_t *k_dev, int64_t n_frames, int32_t H, int32_t W,
                      int32_t block_size, int32_t Q, uint32_t flags, uint8_t *rgb_dev,
                      void *stream);

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

#ifdef __cplusplus
}
#endif
#endif /* VCF_AMD_H */
