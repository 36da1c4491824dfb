#!/usr/bin/env python3
"""Device time of the training head's dW im2col variants on the step's shapes (HIP events, 50 launches each):
tap-major mmt_im2col3x3_up_bf16 vs channel-major mmt_im2col3x3_cm_bf16 (LDS-staged transpose)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "multi-modal-tracking_amd"))
import torch  # noqa: E402
from mmt_amd._lib import LIB, check  # noqa: E402

SHAPES = [(16, 20, 768, 1), (16, 20, 384, 1), (16, 40, 192, 2), (16, 80, 96, 2), (16, 40, 96, 1), (16, 80, 48, 1)]


def main():
    st = torch.cuda.current_stream().cuda_stream
    for B, H, C, up in SHAPES:
        x = torch.randn(B, H // up, H // up, C, device="cuda").bfloat16()
        out = torch.empty(B * H * H, 9 * C, device="cuda", dtype=torch.bfloat16)
        res = []
        for name, fn in (("tap", LIB.mmt_im2col3x3_up_bf16), ("cm", LIB.mmt_im2col3x3_cm_bf16)):
            for _ in range(3):
                check(fn(x.data_ptr(), out.data_ptr(), B, H, H, C, up, st), name)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(50):
                check(fn(x.data_ptr(), out.data_ptr(), B, H, H, C, up, st), name)
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / 50
            res.append("%s %.1f us (%.2f TB/s written)" % (name, us, out.numel() * 2 / us / 1e6))
        print("B=%d H=%d C=%d up=%d: %s" % (B, H, C, up, "; ".join(res)))


if __name__ == "__main__":
    main()
