// Generic NHWC layer kernels (ops_generic.hip).
#pragma once
#include <hip/hip_runtime.h>

namespace gops {

struct ConvShape {
  int N, H, W, C;  // input
  int K;           // output channels
  int R, S;        // kernel
  int stride, pad;
  int OH, OW;
};

struct PoolShape {
  int N, H, W, C, k, stride, pad, OH, OW;
};

void conv_fwd(const ConvShape& s, const float* x, const float* w, const float* bias, float* y,
              bool relu, hipStream_t st);
void conv_bwd_data(const ConvShape& s, const float* dy, const float* w, float* dx, hipStream_t st);
int conv_filter_splits(const ConvShape& s);
// part: workspace of conv_filter_splits(s) * R*S*C*K floats; dw written (not accumulated)
void conv_bwd_filter(const ConvShape& s, const float* x, const float* dy, float* part, float* dw,
                     hipStream_t st);
// mode 0: s1 = colsum(a), s2 = colsum(a^2); mode 1: s1 = colsum(a), s2 = colsum(a*b)
void colsum2(const float* a, const float* b, long long rows, int C, float* s1, float* s2, int mode,
             hipStream_t st);
void bn_fwd(const float* x, long long rows, int C, const float* g, const float* b,
            const float* res, float* y, float* mean, float* rstd, float* sum, float* sumsq,
            float eps, bool relu, bool training, const float* rmean, const float* rvar,
            hipStream_t st);
void bn_bwd(const float* x, const float* dy, const float* y, const float* mean, const float* rstd,
            const float* g, long long rows, int C, bool relu, float* dym, float* xh, float* dg,
            float* db, float* dx, float* dres, hipStream_t st);
void maxpool_fwd(const PoolShape& p, const float* x, float* y, int* arg, hipStream_t st);
void maxpool_bwd(const PoolShape& p, const float* dy, const int* arg, float* dx, hipStream_t st);
void avgpool_fwd(const float* x, float* y, int N, int HW, int C, hipStream_t st);
void avgpool_bwd(const float* dy, float* dx, int N, int HW, int C, hipStream_t st);
void xent(const float* logits, const int* labels, int B, int C, float* loss_rows, float* dlogits,
          int* correct, hipStream_t st);
void relu_bwd(const float* dy, const float* y, float* dx, long long n, hipStream_t st);
void lr_from_step(const long long* step, int n_local, int batch, float base, float decay,
                  float* lr, hipStream_t st);
void gather_batch(const float* data, const int* labels, const long long* step, int n_local,
                  int batch, long long row_elems, float* xb, int* yb, hipStream_t st);

}  // namespace gops
