// bf16 instances of the blocked implicit-GEMM convolution (bconv_kernel.h)
// with 2 16-byte channel group(s) per lane group: one translation unit per
// (element type, CV) so the instances compile in parallel.
#include "bconv_kernel.h"

namespace hcu {

template <>
bool bconv_launch_cv<uint16_t, 2>(const GConvArgs &a, hipStream_t s, const dim3 &grid, double fl, double by) {
  BCONV_CV_BODY(uint16_t, "bf16", 2)
}

}  // namespace hcu
