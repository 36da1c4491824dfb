// Tracker-side pre/post-processing on the GPU.
//
//   mmt_sample_target   sample_target (lib/train/data/processing_utils.py:15-77: square crop of
//                       area factor^2 * w*h centred on the box, zero padding, cv2.resize to
//                       output_sz) followed by the tracker's preprocessor
//                       (lib/test/tracker/tracker_utils.py:24-48: optional cv2.applyColorMap for the
//                       TIR crop, HWC uint8 -> CHW fp32, /255, -mean, /std), straight into the
//                       model's fp32 input buffer.  The crop box is computed on the device from the
//                       device-resident tracker state, so a tracking step needs no host round trip.
//   mmt_track_update    the per-frame box post-processing of the trackers
//                       (lib/test/tracker/mixformer_vit_rgbt.py:92-95, :124-131: scale the predicted
//                       cxcywh back to image pixels, map_box_back, lib/utils/box_ops.py:155-164
//                       clip_box with margin 10), updating the device-resident state in place.
//
// cv2 is not part of this image, so the resize arithmetic restates OpenCV's 8-bit INTER_LINEAR
// path (imgproc resize.cpp: float source coordinate (d+0.5)*scale-0.5, 11-bit fixed-point weights
// rounded half-to-even, the horizontal pass in int, the vertical pass as VResizeLinearVec_32s8u
// computes it: ((h0>>4)*b0>>16) + ((h1>>4)*b1>>16), +2, >>2, saturate; rows clamped, columns past
// the edges taken with weight 2048) and its exact-2x INTER_AREA shortcut ((a+b+c+d+2)>>2); the
// colour map is cvtColor(BGR2GRAY) fixed point (1868, 9617, 4899, >>14) then a 256x3 LUT passed in.
// The oracle (oracle/preprocess.py) restates the same arithmetic; both are bit-exact to each other.
#include "common.hpp"

// Parity is bit-exact against separately rounded torch / numpy / Python ops: no FMA contraction.
#pragma clang fp contract(off)

namespace {

struct CropBatch {
    mmt_crop_params c[MMT_MAX_CROPS];
};

// Python's int(round(v)) for the crop corner: round half to even.
MMT_DEV int py_round(double v) { return (int)rint(v); }

MMT_DEV int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

MMT_DEV short coef(float v) {  // saturate_cast<short>(v * INTER_RESIZE_COEF_SCALE): cvRound
    const int r = (int)rintf(v * 2048.f);
    return (short)clampi(r, -32768, 32767);
}

struct Geo {
    int x1, y1, crop, xlim, ylim;  // padded-crop origin, size, and the first image column/row not copied
};

MMT_DEV Geo crop_geometry(const mmt_crop_params& p) {
    const double x = p.box[0], y = p.box[1], w = p.box[2], h = p.box[3];
    Geo g;
    g.crop = (int)ceil(sqrt(w * h) * p.factor);
    g.x1 = py_round(x + 0.5 * w - g.crop * 0.5);
    g.y1 = py_round(y + 0.5 * h - g.crop * 0.5);
    // im[y1+y1_pad : y2-y2_pad, x1+x1_pad : x2-x2_pad] with x2_pad = max(x2 - W + 1, 0): when the crop
    // runs past the right (bottom) edge, the last image column (row) is not copied either.
    const int x2 = g.x1 + g.crop, y2 = g.y1 + g.crop;
    g.xlim = x2 >= p.W ? p.W - 1 : p.W;
    g.ylim = y2 >= p.H ? p.H - 1 : p.H;
    return g;
}

// padded crop pixel (row r, col c) channel ch: image pixel or the constant border 0
MMT_DEV int src_px(const mmt_crop_params& p, const Geo& g, int r, int c, int ch) {
    const int iy = g.y1 + r, ix = g.x1 + c;
    if (iy < 0 || ix < 0 || iy >= g.ylim || ix >= g.xlim) return 0;
    return p.image[((int64_t)iy * p.W + ix) * 3 + ch];
}

__global__ __launch_bounds__(256) void sample_target_kernel(const CropBatch cb) {
    const mmt_crop_params& p = cb.c[blockIdx.y];
    const int os = p.out_sz;
    const int idx = blockIdx.x * 256 + threadIdx.x;
    if (idx >= os * os) return;
    const int dy = idx / os, dx = idx - dy * os;
    const Geo g = crop_geometry(p);
    if (idx == 0 && p.crop) {
        p.crop[0] = g.x1;
        p.crop[1] = g.y1;
        p.crop[2] = g.crop;
        p.crop[3] = (double)os / g.crop;  // resize_factor = output_sz / crop_sz
    }
    int v[3] = {0, 0, 0};
    if (g.crop >= 1) {
        const double inv = (double)os / g.crop, scale = 1.0 / inv;
        const int is = (int)rint(scale);
        if (is == 2 && fabs(scale - is) < 2.220446049250313e-16) {  // INTER_LINEAR at exactly 1/2 -> INTER_AREA
#pragma unroll
            for (int ch = 0; ch < 3; ++ch)
                v[ch] = (src_px(p, g, 2 * dy, 2 * dx, ch) + src_px(p, g, 2 * dy, 2 * dx + 1, ch) +
                         src_px(p, g, 2 * dy + 1, 2 * dx, ch) + src_px(p, g, 2 * dy + 1, 2 * dx + 1, ch) + 2) >> 2;
        } else {
            float fx = (float)((dx + 0.5) * scale - 0.5);
            int sx = (int)floorf(fx);
            fx -= sx;
            if (sx < 0) fx = 0.f, sx = 0;
            if (sx >= g.crop - 1) fx = 0.f, sx = g.crop - 1;
            float fy = (float)((dy + 0.5) * scale - 0.5);
            const int sy = (int)floorf(fy);
            fy -= sy;
            const int a0 = coef(1.f - fx), a1 = coef(fx), b0 = coef(1.f - fy), b1 = coef(fy);
            const int r0 = clampi(sy, 0, g.crop - 1), r1 = clampi(sy + 1, 0, g.crop - 1);
            const int sx1 = min(sx + 1, g.crop - 1);  // weight a1 is 0 whenever sx + 1 is past the edge
#pragma unroll
            for (int ch = 0; ch < 3; ++ch) {
                const int h0 = src_px(p, g, r0, sx, ch) * a0 + src_px(p, g, r0, sx1, ch) * a1;
                const int h1 = src_px(p, g, r1, sx, ch) * a0 + src_px(p, g, r1, sx1, ch) * a1;
                const int t = (((h0 >> 4) * b0) >> 16) + (((h1 >> 4) * b1) >> 16);
                v[ch] = clampi((t + 2) >> 2, 0, 255);
            }
        }
    }
    const int64_t o = (int64_t)dy * os + dx;
    if (p.patch) {
#pragma unroll
        for (int ch = 0; ch < 3; ++ch) p.patch[o * 3 + ch] = (uint8_t)v[ch];
    }
    if (p.lut) {  // cv2.applyColorMap on a 3-channel crop: BGR2GRAY, GRAY2BGR, per-channel LUT
        const int gray = (v[0] * 1868 + v[1] * 9617 + v[2] * 4899 + (1 << 13)) >> 14;
#pragma unroll
        for (int ch = 0; ch < 3; ++ch) v[ch] = p.lut[gray * 3 + ch];
    }
    if (p.out) {
        const float inv255 = 1.0f / 255.0f;  // torch: tensor / python scalar = tensor * (1 / scalar)
#pragma unroll
        for (int ch = 0; ch < 3; ++ch) p.out[(int64_t)ch * os * os + o] = ((float)v[ch] * inv255 - p.mean[ch]) / p.std[ch];
    }
}

__global__ void track_update_kernel(const float* __restrict__ pred, const double* __restrict__ crop,
                                    double* __restrict__ state, int n, int H, int W, int search_size, double margin) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double rf = crop[i * 4 + 3];
    const float inv = 1.0f / (float)rf;  // torch: fp32 tensor / python float = tensor * (1 / (float)scalar)
    double b[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) b[j] = (double)((pred[i * 4 + j] * (float)search_size) * inv);
    double* s = state + i * 4;
    const double cx_prev = s[0] + 0.5 * s[2], cy_prev = s[1] + 0.5 * s[3];
    const double half = 0.5 * search_size / rf;
    const double cx = b[0] + (cx_prev - half), cy = b[1] + (cy_prev - half);
    double x1 = cx - 0.5 * b[2], y1 = cy - 0.5 * b[3];
    double x2 = x1 + b[2], y2 = y1 + b[3];
    x1 = fmin(fmax(0.0, x1), W - margin);
    x2 = fmin(fmax(margin, x2), (double)W);
    y1 = fmin(fmax(0.0, y1), H - margin);
    y2 = fmin(fmax(margin, y2), (double)H);
    s[0] = x1;
    s[1] = y1;
    s[2] = fmax(margin, x2 - x1);
    s[3] = fmax(margin, y2 - y1);
}

}  // namespace

extern "C" int mmt_sample_target(const mmt_crop_params* p, int n, void* stream) {
    if (!p || n <= 0 || n > MMT_MAX_CROPS) return MMT_EBADARG;
    CropBatch cb;
    int os = 0;
    for (int i = 0; i < n; ++i) {
        const mmt_crop_params& c = p[i];
        if (!c.image || !c.box || c.H <= 0 || c.W <= 0 || c.out_sz <= 0 || !(c.factor > 0.0)) return MMT_EBADARG;
        if (!c.out && !c.patch) return MMT_EBADARG;
        if (i > 0 && c.out_sz != os) return MMT_EBADARG;  // one grid per launch
        os = c.out_sz;
        cb.c[i] = c;
    }
    dim3 grid((os * os + 255) / 256, n);
    hipLaunchKernelGGL(sample_target_kernel, grid, dim3(256), 0, (hipStream_t)stream, cb);
    return launch_status();
}

extern "C" int mmt_track_update(const float* pred_cxcywh, const double* crop, double* state, int n, int H, int W,
                                int search_size, double margin, void* stream) {
    if (!pred_cxcywh || !crop || !state || n <= 0 || H <= 0 || W <= 0 || search_size <= 0) return MMT_EBADARG;
    hipLaunchKernelGGL(track_update_kernel, dim3((n + 63) / 64), dim3(64), 0, (hipStream_t)stream, pred_cxcywh, crop,
                       state, n, H, W, search_size, margin);
    return launch_status();
}
