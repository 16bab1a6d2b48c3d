// kernels_pre.hip -- image preprocessing on the GPU:
// processing_paligemma.py:13-18,40-49 = PIL Image.resize(BICUBIC) -> x/255 -> (x-0.5)/0.5 -> CHW.
//
// PIL's resample (libImaging/Resample.c; restated in oracle/resize_np.py) is reproduced
// bit-exactly: per-output-index coefficients in double (bicubic a = -0.5, support 2 x
// max(scale, 1), taps [int(c - s + .5), int(c + s + .5)) normalised by their sum), converted to
// 22-bit fixed point rounding half away from zero; a horizontal pass over only the source rows
// the vertical pass uses, to a uint8 image (clip8 of (sum + 2^21) >> 22), then the vertical
// pass.  The vertical pass also applies the reference's rescale / normalize / transpose:
// float((double)u8 * (1/255)) then (x - 0.5f) / 0.5f, written as float32 CHW.
#include <cmath>

#include "common.h"
#include "launch.h"

namespace pgmi {

constexpr int kPrePrec = 32 - 8 - 2;

__device__ __forceinline__ double pre_bicubic(double x) {
    const double a = -0.5;
    if (x < 0.0) x = -x;
    if (x < 1.0) return ((a + 2.0) * x - (a + 3.0)) * x * x + 1;
    if (x < 2.0) return (((x - 5) * x + 8) * x - 4) * a;
    return 0.0;
}

// one thread per output index of one axis: bounds (xmin, n) and n fixed-point weights
__global__ void k_pre_coeffs(int in_size, int out_size, int ksize, int2* __restrict__ bounds,
                             int* __restrict__ kk) {
    const int xx = blockIdx.x * blockDim.x + threadIdx.x;
    if (xx >= out_size) return;
    const double scale = (double)in_size / out_size;
    const double filterscale = scale < 1.0 ? 1.0 : scale;
    const double support = 2.0 * filterscale;
    const double center = (xx + 0.5) * scale;
    const double ss = 1.0 / filterscale;
    int xmin = (int)(center - support + 0.5);
    if (xmin < 0) xmin = 0;
    int xmax = (int)(center + support + 0.5);
    if (xmax > in_size) xmax = in_size;
    xmax -= xmin;
    double ww = 0.0;
    for (int x = 0; x < xmax; ++x) ww += pre_bicubic((x + xmin - center + 0.5) * ss);
    int* k = kk + (long)xx * ksize;
    for (int x = 0; x < ksize; ++x) {
        double w = x < xmax ? pre_bicubic((x + xmin - center + 0.5) * ss) : 0.0;
        if (x < xmax && ww != 0.0) w /= ww;
        k[x] = x < xmax ? (w < 0 ? (int)(-0.5 + w * (1 << kPrePrec)) : (int)(0.5 + w * (1 << kPrePrec))) : 0;
    }
    bounds[xx] = make_int2(xmin, xmax);
}

__device__ __forceinline__ uint8_t pre_clip8(int acc) {
    if (acc >= (1 << kPrePrec << 8)) return 255;
    if (acc <= 0) return 0;
    return (uint8_t)(acc >> kPrePrec);
}

__device__ __forceinline__ float pre_norm(uint8_t v) {
    const float f = (float)((double)v * (1.0 / 255.0));  // rescale: float64 product, cast (:20-23)
    return (f - 0.5f) / 0.5f;                             // normalize in float32 (:25-29)
}

// horizontal pass: rows [0, rows) of src (already offset to the first used row) -> tmp uint8
// [rows][out_w][3]; one thread per output pixel (3 channels)
__global__ void k_pre_h(const uint8_t* __restrict__ src, int src_w, int rows, int out_w, int ksize,
                        const int2* __restrict__ bounds, const int* __restrict__ kk, uint8_t* __restrict__ tmp) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (long)rows * out_w) return;
    const int y = (int)(i / out_w), xx = (int)(i % out_w);
    const int2 bd = bounds[xx];
    const int* k = kk + (long)xx * ksize;
    const uint8_t* p = src + ((long)y * src_w + bd.x) * 3;
    int s0 = 1 << (kPrePrec - 1), s1 = s0, s2 = s0;
    for (int x = 0; x < bd.y; ++x) {
        const int w = k[x];
        s0 += p[3 * x + 0] * w;
        s1 += p[3 * x + 1] * w;
        s2 += p[3 * x + 2] * w;
    }
    uint8_t* o = tmp + i * 3;
    o[0] = pre_clip8(s0);
    o[1] = pre_clip8(s1);
    o[2] = pre_clip8(s2);
}

// vertical pass (or a plain copy when the height is unchanged) + rescale/normalize -> CHW f32
__global__ void k_pre_v(const uint8_t* __restrict__ img, int w, int out_h, int ksize, int identity,
                        const int2* __restrict__ bounds, const int* __restrict__ kk, float* __restrict__ out) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (long)out_h * w) return;
    const int yy = (int)(i / w), x = (int)(i % w);
    uint8_t v[3];
    if (identity) {
        const uint8_t* p = img + ((long)yy * w + x) * 3;
        v[0] = p[0]; v[1] = p[1]; v[2] = p[2];
    } else {
        const int2 bd = bounds[yy];
        const int* k = kk + (long)yy * ksize;
        int s0 = 1 << (kPrePrec - 1), s1 = s0, s2 = s0;
        for (int y = 0; y < bd.y; ++y) {
            const uint8_t* p = img + ((long)(bd.x + y) * w + x) * 3;
            const int wk = k[y];
            s0 += p[0] * wk;
            s1 += p[1] * wk;
            s2 += p[2] * wk;
        }
        v[0] = pre_clip8(s0); v[1] = pre_clip8(s1); v[2] = pre_clip8(s2);
    }
    const long plane = (long)out_h * w;
#pragma unroll
    for (int c = 0; c < 3; ++c) out[c * plane + i] = pre_norm(v[c]);
}

static int pre_ksize(int in_size, int out_size) {
    const double scale = (double)in_size / out_size;
    const double support = 2.0 * (scale < 1.0 ? 1.0 : scale);
    return (int)std::ceil(support) * 2 + 1;
}

// host mirror of the first / last source row the vertical pass reads (Resample.c ybox_first/last)
static void pre_row_range(int in_h, int out_h, int* y0, int* y1) {
    const double scale = (double)in_h / out_h;
    const double support = 2.0 * (scale < 1.0 ? 1.0 : scale);
    auto lo = [&](int yy) {
        const double c = (yy + 0.5) * scale;
        int m = (int)(c - support + 0.5);
        return m < 0 ? 0 : m;
    };
    auto hi = [&](int yy) {
        const double c = (yy + 0.5) * scale;
        int m = (int)(c + support + 0.5);
        return m > in_h ? in_h : m;
    };
    *y0 = lo(0);
    *y1 = hi(out_h - 1);
}

size_t preprocess_scratch_bytes(int H, int W, int out_h, int out_w) {
    const int kh = pre_ksize(W, out_w), kv = pre_ksize(H, out_h);
    const size_t coef = (size_t)out_w * (8 + 4 * kh) + (size_t)out_h * (8 + 4 * kv);
    return coef + (size_t)H * out_w * 3 + 256;
}

void preprocess(hipStream_t s, const uint8_t* src, int H, int W, int out_h, int out_w, float* out, void* scratch) {
    const int kh = pre_ksize(W, out_w), kv = pre_ksize(H, out_h);
    uint8_t* sp = reinterpret_cast<uint8_t*>(scratch);
    int2* bh = reinterpret_cast<int2*>(sp);
    int2* bv = bh + out_w;
    int* kkh = reinterpret_cast<int*>(bv + out_h);
    int* kkv = kkh + (long)out_w * kh;
    uint8_t* tmp = reinterpret_cast<uint8_t*>(kkv + (long)out_h * kv);
    const bool need_h = out_w != W, need_v = out_h != H;
    hipLaunchKernelGGL(k_pre_coeffs, dim3((out_w + 127) / 128), dim3(128), 0, s, W, out_w, kh, bh, kkh);
    hipLaunchKernelGGL(k_pre_coeffs, dim3((out_h + 127) / 128), dim3(128), 0, s, H, out_h, kv, bv, kkv);
    int y0 = 0, y1 = H;
    if (need_v) pre_row_range(H, out_h, &y0, &y1);
    const uint8_t* img = src;  // rows addressed by absolute source row (the vertical bounds)
    if (need_h) {
        const long n = (long)(y1 - y0) * out_w;
        hipLaunchKernelGGL(k_pre_h, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, src + (long)y0 * W * 3, W,
                           y1 - y0, out_w, kh, bh, kkh, tmp);
        img = tmp - (long)y0 * out_w * 3;  // tmp row r holds source row y0 + r
    }
    const long n = (long)out_h * out_w;
    hipLaunchKernelGGL(k_pre_v, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, img, out_w, out_h, kv,
                       need_v ? 0 : 1, bv, kkv, out);
}

}  // namespace pgmi
