/* CPU restatement of the IPP temporal tools of the reference (src/IPP_DCT.py).
 *
 * TEST INFRASTRUCTURE ONLY: the checker for vcf_amd/csrc/vcf_ipp.hip, never
 * the product.  Follows, step for step:
 *   vcfo_ipp_gray          cv2.cvtColor(RGB2GRAY) as called by IPP.block_matching
 *                          (IPP_DCT.py:357-358); OpenCV's fixed-point formula for
 *                          8-bit images, assumption A10 (cv2 absent here: unpinned)
 *   vcfo_ipp_block_match   IPP.block_matching (:344-376) -> _process_block_row
 *                          (:207-246): full search, first strict minimum in
 *                          dy-outer / dx-inner order over in-bounds candidates;
 *                          --fast: _three_step_search (:159-204) with the
 *                          centre moving inside the 3x3 sweep
 *   vcfo_ipp_mc            IPP.motion_compensate (:378-395)
 * Pinned against tests/golden/ipp.npz (those functions executed unmodified).
 */
#include <limits.h>
#include <stdint.h>
#include <stdlib.h>

void vcfo_ipp_gray(const uint8_t *rgb, int64_t n, uint8_t *gray) {
    for (int64_t p = 0; p < n; p++) {
        const uint8_t *q = rgb + 3 * p;
        gray[p] = (uint8_t)((4899 * q[0] + 9617 * q[1] + 1868 * q[2] + 8192) >> 14);
    }
}

/* np.sum(np.abs(curr.astype(int16) - ref.astype(int16))) over a bs x bs block */
static long block_sad(const uint8_t *ref, const uint8_t *cur, int W, int ry, int rx, int cy, int cx, int bs) {
    long s = 0;
    for (int y = 0; y < bs; y++)
        for (int x = 0; x < bs; x++)
            s += labs((long)cur[(long)(cy + y) * W + cx + x] - (long)ref[(long)(ry + y) * W + rx + x]);
    return s;
}

static int inside(int y, int x, int bs, int H, int W) { return y >= 0 && y + bs <= H && x >= 0 && x + bs <= W; }

static void full_search(const uint8_t *rg, const uint8_t *cg, int H, int W, int i, int j, int bs, int sr,
                        int *bx, int *by) {
    long best = LONG_MAX;           /* min_sad = inf */
    *bx = 0;
    *by = 0;
    for (int dy = -sr; dy <= sr; dy++) {
        int ry = i + dy;
        if (ry < 0 || ry + bs > H) continue;
        for (int dx = -sr; dx <= sr; dx++) {
            int rx = j + dx;
            if (rx < 0 || rx + bs > W) continue;
            long s = block_sad(rg, cg, W, ry, rx, i, j, bs);
            if (s < best) {
                best = s;
                *bx = dx;
                *by = dy;
            }
        }
    }
}

static void three_step(const uint8_t *rg, const uint8_t *cg, int H, int W, int i, int j, int bs, int sr,
                       int *bx, int *by) {
    int step = sr / 2;   /* Python // on a non-negative int */
    int cx = j, cy = i;
    *bx = 0;
    *by = 0;
    long best = LONG_MAX;
    if (inside(cy, cx, bs, H, W)) best = block_sad(rg, cg, W, cy, cx, i, j, bs);
    while (step >= 1) {
        int improved = 0;
        for (int a = -1; a <= 1; a++)
            for (int b = -1; b <= 1; b++) {
                if (a == 0 && b == 0) continue;
                int ry = cy + a * step, rx = cx + b * step;
                if (!inside(ry, rx, bs, H, W)) continue;
                long s = block_sad(rg, cg, W, ry, rx, i, j, bs);
                if (s < best) {
                    best = s;
                    *bx = rx - j;
                    *by = ry - i;
                    cx = rx;
                    cy = ry;
                    improved = 1;
                }
            }
        step = improved ? (step / 2 > 1 ? step / 2 : 1) : step / 2;
    }
}

/* mv: (H/bs) x (W/bs) x 2 float32 (dx, dy), as the reference's mv_field */
void vcfo_ipp_block_match(const uint8_t *ref, const uint8_t *cur, int H, int W, int bs, int sr, int fast, float *mv) {
    uint8_t *rg = malloc((size_t)H * W), *cg = malloc((size_t)H * W);
    vcfo_ipp_gray(ref, (int64_t)H * W, rg);
    vcfo_ipp_gray(cur, (int64_t)H * W, cg);
    int nbx = W / bs;
    for (int i = 0; i + bs <= H; i += bs)
        for (int j = 0; j + bs <= W; j += bs) {
            int dx, dy;
            if (fast)
                three_step(rg, cg, H, W, i, j, bs, sr, &dx, &dy);
            else
                full_search(rg, cg, H, W, i, j, bs, sr, &dx, &dy);
            float *m = mv + 2 * ((long)(i / bs) * nbx + j / bs);
            m[0] = (float)dx;
            m[1] = (float)dy;
        }
    free(rg);
    free(cg);
}

void vcfo_ipp_mc(const uint8_t *frame, const float *mv, int H, int W, int bs, uint8_t *out) {
    int nbx = W / bs;
    for (long p = 0; p < (long)H * W * 3; p++) out[p] = 0;   /* np.zeros_like */
    for (int i = 0; i + bs <= H; i += bs)
        for (int j = 0; j + bs <= W; j += bs) {
            const float *m = mv + 2 * ((long)(i / bs) * nbx + j / bs);
            int ry = (int)(i + m[1]), rx = (int)(j + m[0]);   /* int() truncates */
            if (!inside(ry, rx, bs, H, W)) {
                ry = i;
                rx = j;
            }
            for (int y = 0; y < bs; y++)
                for (int x = 0; x < 3 * bs; x++)
                    out[((long)(i + y) * W + j) * 3 + x] = frame[((long)(ry + y) * W + rx) * 3 + x];
        }
}
