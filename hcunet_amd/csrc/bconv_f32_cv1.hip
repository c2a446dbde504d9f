// f32 instances of the blocked implicit-GEMM convolution (bconv_kernel.h)
// with 1 16-byte channel group(s) per lane group: one translation unit per
// (element type, CV) so the instances compile in parallel.
#include "bconv_kernel.h"

namespace hcu {

template <>
bool bconv_launch_cv<float, 1>(const GConvArgs &a, hipStream_t s, const dim3 &grid, double fl, double by) {
  BCONV_CV_BODY(float, "f32", 1)
}

}  // namespace hcu
