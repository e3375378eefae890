// vcf_inflate_wincheck.hip -- the GPU inflate (csrc/vcf_inflate.hip) built as
// its window-check diagnostic for the A/B library: vcf_inflate_strips_wincheck
// decodes exactly as vcf_inflate_strips and also counts, per strip, every read
// of the 32 KiB output ring that falls outside the ring's valid span (a
// back-reference byte not yet written or already overwritten, a flush of bytes
// no longer in the ring).  tests/test_inflate_gpu.py runs it and expects zero.
#define VCF_INFLATE_WINCHECK_BUILD 1
#include "vcf_inflate.hip"
