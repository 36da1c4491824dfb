// The training step's corner read-out and box loss, forward and backward, replacing ~100 small
// PyTorch launches per step with four:
//
//   mmt_corner_boxes   Pyramid_Corner_Predictor.soft_argmax of both corner score maps (head.py:200-212) and
//                      the normalisation to [0, 1] (head.py:176-177): xyxy[b] = (E_tl[x], E_tl[y], E_br[x], E_br[y]) *
//                      (1 / img_sz), E[.] under softmax(score) over the fh x fh map, coordinates stride * (col, row);
//                      backward: d score_k = p_k (gx (x_k - E[x]) + gy (y_k - E[y])) (the softmax backward of the
//                      expectation's gradient)
//   mmt_box_loss       MixFormerRGBTActor.compute_losses (actors/mixformer_rgbt.py:127-168) with the CIoU of
//                      lib/utils/box_ops.py:100-152: pred cxcywh -> xyxy, gt xywh -> xyxy clamped to [0, 1],
//                      loss = iou_w mean(1 - clamp(iou - u - alpha v, -1, 1)) + l1_w mean|pred - gt|, alpha without
//                      gradient; outputs (loss, ciou loss, l1, mean iou); backward: d pred from d loss, the same
//                      chain autograd builds (min / max ties split the gradient in halves, clamps pass it at their
//                      bounds inclusive, sign(0) = 0 in the L1 term).
//
// fp32 throughout; the sums run in a fixed order (bitwise reproducible).
#include "common.hpp"

// each operation rounded on its own, as PyTorch's separate elementwise kernels round it (no fused multiply-adds)
#pragma clang fp contract(off)

namespace {

constexpr int CB_T = 256;

// one workgroup per sample: both corners' softmax statistics and expectations
__global__ __launch_bounds__(CB_T) void corner_boxes_kernel(const float* __restrict__ tl, const float* __restrict__ br,
                                                            float* __restrict__ xyxy, float* __restrict__ stats, int fh,
                                                            float stride, float inv_img) {
    __shared__ float red[CB_T / 64];
    const int b = blockIdx.x, n = fh * fh;
    for (int c = 0; c < 2; ++c) {
        const float* s = (c == 0 ? tl : br) + (int64_t)b * n;
        float mx = -INFINITY;
        for (int k = threadIdx.x; k < n; k += CB_T) mx = fmaxf(mx, s[k]);
        mx = block_max<CB_T>(mx, red);
        float se = 0.f;
        for (int k = threadIdx.x; k < n; k += CB_T) se += expf(s[k] - mx);
        se = block_sum<CB_T>(se, red);
        float ex = 0.f, ey = 0.f;
        for (int k = threadIdx.x; k < n; k += CB_T) {
            const float p = expf(s[k] - mx) / se;
            ex += stride * (float)(k % fh) * p;
            ey += stride * (float)(k / fh) * p;
        }
        ex = block_sum<CB_T>(ex, red);
        ey = block_sum<CB_T>(ey, red);
        if (threadIdx.x == 0) {
            xyxy[b * 4 + 2 * c] = ex * inv_img;
            xyxy[b * 4 + 2 * c + 1] = ey * inv_img;
            float* st = stats + (b * 2 + c) * 4;
            st[0] = mx, st[1] = se, st[2] = ex, st[3] = ey;
        }
    }
}

__global__ __launch_bounds__(CB_T) void corner_boxes_bwd_kernel(const float* __restrict__ tl, const float* __restrict__ br,
                                                                const float* __restrict__ stats,
                                                                const float* __restrict__ dxyxy, float* __restrict__ dtl,
                                                                float* __restrict__ dbr, int fh, float stride,
                                                                float inv_img) {
    const int b = blockIdx.x, c = blockIdx.y, n = fh * fh;
    const float* s = (c == 0 ? tl : br) + (int64_t)b * n;
    float* d = (c == 0 ? dtl : dbr) + (int64_t)b * n;
    const float* st = stats + (b * 2 + c) * 4;
    const float mx = st[0], se = st[1], ex = st[2], ey = st[3];
    const float gx = dxyxy[b * 4 + 2 * c] * inv_img, gy = dxyxy[b * 4 + 2 * c + 1] * inv_img;
    for (int k = threadIdx.x; k < n; k += CB_T) {
        const float p = expf(s[k] - mx) / se;
        d[k] = p * (gx * (stride * (float)(k % fh) - ex) + gy * (stride * (float)(k / fh) - ey));
    }
}

// ---- box loss ----
struct BoxTerms {  // one sample's CIoU / L1 terms and what the backward needs
    float b1[4], b2[4];
    float w1, h1, w2, h2, c1x, c1y, c2x, c2y;
    float lo1[2], hi1[2], lo2[2], hi2[2];
    float mi[2], ma[2];  // min(hi1, hi2) - max(lo1, lo2), max(hi1, hi2) - min(lo1, lo2)
    float iw[2], ew[2];  // clamp(mi, 0), clamp(ma, 0)
    float inter, inter_diag, c_diag, uni, u, iou, at, v, alpha, raw, cious;
};

// torch.clamp: NaN stays NaN (fminf / fmaxf would drop it)
MMT_DEV float clampf(float x, float lo, float hi) { return x != x ? x : fminf(fmaxf(x, lo), hi); }
MMT_DEV float clamp_lo(float x, float lo) { return x != x ? x : fmaxf(x, lo); }

MMT_DEV void box_terms(const float* pred, const float* gt, BoxTerms& t) {
    // pred cxcywh -> xyxy (mixformer_rgbt.py: box_cxcywh_to_xyxy); gt xywh -> xyxy clamped (box_xywh_to_xyxy)
    t.b1[0] = pred[0] - 0.5f * pred[2];
    t.b1[1] = pred[1] - 0.5f * pred[3];
    t.b1[2] = pred[0] + 0.5f * pred[2];
    t.b1[3] = pred[1] + 0.5f * pred[3];
    t.b2[0] = clampf(gt[0], 0.f, 1.f);
    t.b2[1] = clampf(gt[1], 0.f, 1.f);
    t.b2[2] = clampf(gt[0] + gt[2], 0.f, 1.f);
    t.b2[3] = clampf(gt[1] + gt[3], 0.f, 1.f);
    t.w1 = t.b1[2] - t.b1[0], t.h1 = t.b1[3] - t.b1[1];
    t.w2 = t.b2[2] - t.b2[0], t.h2 = t.b2[3] - t.b2[1];
    t.c1x = (t.b1[0] + t.b1[2]) / 2.f, t.c1y = (t.b1[1] + t.b1[3]) / 2.f;
    t.c2x = (t.b2[0] + t.b2[2]) / 2.f, t.c2y = (t.b2[1] + t.b2[3]) / 2.f;
    const float wh1[2] = {t.w1, t.h1}, wh2[2] = {t.w2, t.h2}, c1[2] = {t.c1x, t.c1y}, c2[2] = {t.c2x, t.c2y};
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        t.lo1[j] = c1[j] - wh1[j] / 2.f, t.hi1[j] = c1[j] + wh1[j] / 2.f;
        t.lo2[j] = c2[j] - wh2[j] / 2.f, t.hi2[j] = c2[j] + wh2[j] / 2.f;
        t.mi[j] = fminf(t.hi1[j], t.hi2[j]) - fmaxf(t.lo1[j], t.lo2[j]);
        t.ma[j] = fmaxf(t.hi1[j], t.hi2[j]) - fminf(t.lo1[j], t.lo2[j]);
        t.iw[j] = clamp_lo(t.mi[j], 0.f);
        t.ew[j] = clamp_lo(t.ma[j], 0.f);
    }
    t.inter = t.iw[0] * t.iw[1];
    const float dx = t.c2x - t.c1x, dy = t.c2y - t.c1y;
    t.inter_diag = dx * dx + dy * dy;
    t.c_diag = t.ew[0] * t.ew[0] + t.ew[1] * t.ew[1];
    t.uni = t.w1 * t.h1 + t.w2 * t.h2 - t.inter;
    t.u = t.inter_diag / t.c_diag;
    t.iou = t.inter / t.uni;
    t.at = atanf(t.w2 / t.h2) - atanf(t.w1 / t.h1);
    t.v = (float)(4.0 / (M_PI * M_PI)) * (t.at * t.at);
    t.alpha = (t.iou > 0.5f ? 1.f : 0.f) * t.v / (1.f - t.iou + t.v);
    t.raw = t.iou - t.u - t.alpha * t.v;
    t.cious = clampf(t.raw, -1.f, 1.f);
}

// d(min(a, b)) / da as torch's minimum backward: 1 where a < b, 1/2 on ties, else 0 (max likewise)
MMT_DEV float dmin_a(float a, float b) { return a < b ? 1.f : (a == b ? 0.5f : 0.f); }
MMT_DEV float dmax_a(float a, float b) { return a > b ? 1.f : (a == b ? 0.5f : 0.f); }
MMT_DEV float sgnf(float x) { return x > 0.f ? 1.f : (x < 0.f ? -1.f : 0.f); }

constexpr int BL_T = 256;

__global__ __launch_bounds__(BL_T) void box_loss_kernel(const float* __restrict__ pred, const float* __restrict__ gt,
                                                        float* __restrict__ out, int B, float iou_w, float l1_w) {
    __shared__ float red[BL_T / 64];
    float s_ciou = 0.f, s_l1 = 0.f, s_iou = 0.f;
    for (int b = threadIdx.x; b < B; b += BL_T) {
        BoxTerms t;
        box_terms(pred + 4 * b, gt + 4 * b, t);
        s_ciou += 1.f - t.cious;
        s_iou += t.iou;
#pragma unroll
        for (int j = 0; j < 4; ++j) s_l1 += fabsf(t.b1[j] - t.b2[j]);
    }
    s_ciou = block_sum<BL_T>(s_ciou, red);
    s_l1 = block_sum<BL_T>(s_l1, red);
    s_iou = block_sum<BL_T>(s_iou, red);
    if (threadIdx.x == 0) {
        const float ciou = s_ciou / (float)B, l1 = s_l1 / (float)(4 * B);
        out[0] = iou_w * ciou + l1_w * l1;
        out[1] = ciou;
        out[2] = l1;
        out[3] = s_iou / (float)B;
    }
}

// d pred (cxcywh) of loss = iou_w mean(1 - cious) + l1_w mean|b1 - b2|, times the incoming d loss
__global__ __launch_bounds__(BL_T) void box_loss_bwd_kernel(const float* __restrict__ pred, const float* __restrict__ gt,
                                                            const float* __restrict__ dloss, float* __restrict__ dpred,
                                                            int B, float iou_w, float l1_w) {
    const int b = blockIdx.x * BL_T + threadIdx.x;
    if (b >= B) return;
    BoxTerms t;
    box_terms(pred + 4 * b, gt + 4 * b, t);
    const float g = dloss[0];
    // d cious: the mean of (1 - cious) times iou_w; clamp passes it on [-1, 1]
    const float dc = (t.raw >= -1.f && t.raw <= 1.f) ? -iou_w * g / (float)B : 0.f;
    const float diou = dc, du = -dc, dv = -t.alpha * dc;
    // u = inter_diag / c_diag
    const float d_idiag = du / t.c_diag, d_cdiag = -du * t.inter_diag / (t.c_diag * t.c_diag);
    // iou = inter / union; union = w1 h1 + w2 h2 - inter
    float dinter = diou / t.uni;
    const float duni = -diou * t.inter / (t.uni * t.uni);
    dinter -= duni;
    float dw1 = duni * t.h1, dh1 = duni * t.w1;
    // v = 4 / pi^2 (atan(w2 / h2) - atan(w1 / h1))^2
    {
        const float da1 = dv * (float)(4.0 / (M_PI * M_PI)) * 2.f * t.at * -1.f;  // d atan(w1 / h1)
        const float r = t.w1 / t.h1, dr = da1 / (1.f + r * r);
        dw1 += dr / t.h1;
        dh1 += -dr * t.w1 / (t.h1 * t.h1);
    }
    // inter = iw0 iw1, c_diag = ew0^2 + ew1^2 (clamps at 0 pass the gradient where the argument >= 0)
    float dhi1[2], dlo1[2];
    const float diw[2] = {dinter * t.iw[1], dinter * t.iw[0]};
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const float dmi = t.mi[j] >= 0.f ? diw[j] : 0.f;
        const float dma = t.ma[j] >= 0.f ? d_cdiag * 2.f * t.ew[j] : 0.f;
        dhi1[j] = dmi * dmin_a(t.hi1[j], t.hi2[j]) + dma * dmax_a(t.hi1[j], t.hi2[j]);
        dlo1[j] = -dmi * dmax_a(t.lo1[j], t.lo2[j]) - dma * dmin_a(t.lo1[j], t.lo2[j]);
    }
    // inter_diag = (c2x - c1x)^2 + (c2y - c1y)^2; lo1 = c1 - wh1 / 2, hi1 = c1 + wh1 / 2
    const float dc1x = -2.f * (t.c2x - t.c1x) * d_idiag + dlo1[0] + dhi1[0];
    const float dc1y = -2.f * (t.c2y - t.c1y) * d_idiag + dlo1[1] + dhi1[1];
    dw1 += (dhi1[0] - dlo1[0]) / 2.f;
    dh1 += (dhi1[1] - dlo1[1]) / 2.f;
    // c1 = (b1[:2] + b1[2:]) / 2; wh1 = b1[2:] - b1[:2]; the L1 term
    float db1[4];
    db1[0] = dc1x / 2.f - dw1;
    db1[1] = dc1y / 2.f - dh1;
    db1[2] = dc1x / 2.f + dw1;
    db1[3] = dc1y / 2.f + dh1;
    const float gl = l1_w * g / (float)(4 * B);
#pragma unroll
    for (int j = 0; j < 4; ++j) db1[j] += gl * sgnf(t.b1[j] - t.b2[j]);
    // b1 = [p_xy - p_wh / 2, p_xy + p_wh / 2]
    float* dp = dpred + 4 * b;
    dp[0] = db1[0] + db1[2];
    dp[1] = db1[1] + db1[3];
    dp[2] = 0.5f * (db1[2] - db1[0]);
    dp[3] = 0.5f * (db1[3] - db1[1]);
}

}  // namespace

extern "C" int mmt_corner_boxes(const float* score_tl, const float* score_br, float* xyxy, float* stats, int B, int fh,
                                float stride, float img_sz, void* stream) {
    if (!score_tl || !score_br || !xyxy || !stats || B <= 0 || fh <= 0 || !(img_sz > 0.f)) return MMT_EBADARG;
    hipLaunchKernelGGL(corner_boxes_kernel, dim3((unsigned)B), dim3(CB_T), 0, (hipStream_t)stream, score_tl, score_br,
                       xyxy, stats, fh, stride, 1.f / img_sz);
    return launch_status();
}

extern "C" int mmt_corner_boxes_bwd(const float* score_tl, const float* score_br, const float* stats, const float* dxyxy,
                                    float* dscore_tl, float* dscore_br, int B, int fh, float stride, float img_sz,
                                    void* stream) {
    if (!score_tl || !score_br || !stats || !dxyxy || !dscore_tl || !dscore_br || B <= 0 || fh <= 0 || !(img_sz > 0.f))
        return MMT_EBADARG;
    hipLaunchKernelGGL(corner_boxes_bwd_kernel, dim3((unsigned)B, 2), dim3(CB_T), 0, (hipStream_t)stream, score_tl,
                       score_br, stats, dxyxy, dscore_tl, dscore_br, fh, stride, 1.f / img_sz);
    return launch_status();
}

extern "C" int mmt_box_loss(const float* pred, const float* gt, float* out, int B, float iou_w, float l1_w,
                            void* stream) {
    if (!pred || !gt || !out || B <= 0) return MMT_EBADARG;
    hipLaunchKernelGGL(box_loss_kernel, dim3(1), dim3(BL_T), 0, (hipStream_t)stream, pred, gt, out, B, iou_w, l1_w);
    return launch_status();
}

extern "C" int mmt_box_loss_bwd(const float* pred, const float* gt, const float* dloss, float* dpred, int B, float iou_w,
                                float l1_w, void* stream) {
    if (!pred || !gt || !dloss || !dpred || B <= 0) return MMT_EBADARG;
    hipLaunchKernelGGL(box_loss_bwd_kernel, dim3((unsigned)((B + BL_T - 1) / BL_T)), dim3(BL_T), 0, (hipStream_t)stream,
                       pred, gt, dloss, dpred, B, iou_w, l1_w);
    return launch_status();
}
