// Boundary-history variants of the multi-row blocked kernel (tb3d_mr.h,
// feature bit 8): the core pass of a hybrid run whose stepped shell reads the
// core's face cells at every intermediate level instead of recomputing a band
// of core cells (fdtd3d_amd/models/blocking.py, history shell).  A translation
// unit of its own so it compiles in parallel with yee3d_tb.hip.

#include "tb3d_mr.h"

namespace tb3d {

namespace {
template <int T>
int hist_sel(int fx, const float* const* ein, const float* const* hin, float* const* eout, float* const* hout,
             const float4* ce4, const float4* ch4, const Box3& BE, const Box3& BH, float cb, float db, int nx, int ny,
             int nz, const Box3* b, const Box3& O, int xchunk, const int* src, const TbSrc& sv, const TfDev* tf,
             const float* gtab, float* hist, int hls, hipStream_t s) {
#define MR_ARGS ein, hin, eout, hout, ce4, ch4, BE, BH, cb, db, nx, ny, nz, b, O, xchunk, src, sv, tf, gtab, hist, hls, s
  switch (fx) {
    case 8: return launch_tb_mr<T, 1, 2, 8>(MR_ARGS);
    case 9: return launch_tb_mr<T, 1, 2, 9>(MR_ARGS);
    case 10: return launch_tb_mr<T, 1, 2, 10>(MR_ARGS);
    case 11: return launch_tb_mr<T, 1, 2, 11>(MR_ARGS);
    case 12: return launch_tb_mr<T, 1, 2, 12>(MR_ARGS);
    case 13: return launch_tb_mr<T, 1, 2, 13>(MR_ARGS);
    case 14: return launch_tb_mr<T, 1, 2, 14>(MR_ARGS);
    case 15: return launch_tb_mr<T, 1, 2, 15>(MR_ARGS);
  }
#undef MR_ARGS
  return (int)hipErrorInvalidValue;
}
}  // namespace

int launch_tb_mr_hist(int T, int fx, const float* const* ein, const float* const* hin, float* const* eout,
                      float* const* hout, const float4* ce4, const float4* ch4, const Box3& BE, const Box3& BH,
                      float cb, float db, int nx, int ny, int nz, const Box3* b, const Box3& O, int xchunk,
                      const int* src, const TbSrc& sv, const TfDev* tf, const float* gtab, float* hist, int hls,
                      hipStream_t s) {
#define MR_ARGS fx, ein, hin, eout, hout, ce4, ch4, BE, BH, cb, db, nx, ny, nz, b, O, xchunk, src, sv, tf, gtab, hist, hls, s
  switch (T) {
    case 1: return hist_sel<1>(MR_ARGS);
    case 2: return hist_sel<2>(MR_ARGS);
    case 3: return hist_sel<3>(MR_ARGS);
    case 4: return hist_sel<4>(MR_ARGS);
    case 5: return hist_sel<5>(MR_ARGS);
  }
#undef MR_ARGS
  return (int)hipErrorInvalidValue;
}

}  // namespace tb3d
