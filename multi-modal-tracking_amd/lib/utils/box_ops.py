"""Host box helpers of lib/utils/box_ops.py used around the tracker (the per-frame path runs them
on the device, csrc/preprocess.hip mmt_track_update)."""


def box_xyxy_to_cxcywh(x):
    """box_ops.py:27-32 (torch tensors, last dim 4)."""
    import torch
    x0, y0, x1, y1 = x.unbind(-1)
    return torch.stack([(x0 + x1) / 2, (y0 + y1) / 2, (x1 - x0), (y1 - y0)], dim=-1)


def clip_box(box: list, H, W, margin=0):
    """box_ops.py:155-164: clamp an [x, y, w, h] box into the W x H frame with a margin."""
    x1, y1, w, h = box
    x2, y2 = x1 + w, y1 + h
    x1, x2 = min(max(0, x1), W - margin), min(max(margin, x2), W)
    y1, y2 = min(max(0, y1), H - margin), min(max(margin, y2), H)
    return [x1, y1, max(margin, x2 - x1), max(margin, y2 - y1)]
