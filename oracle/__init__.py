"""ORACLE — TEST INFRASTRUCTURE ONLY.

CPU restatement of the reference's MixFormer RGB-T forward path (LZ-QWQ/Multi-modal-Tracking,
lib/models/mixformer_vit_rgbt/*), used as the parity checker for the HIP path and as the
`cpu_baseline` leg of bench.py.  Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may import it; the product (multi-modal-tracking_amd/) never does.

Pinning: the restatement is checked against golden vectors produced by the reference's own
Python run on CPU under import stubs (tests/golden/make_golden.py), and against the
reference's known-answer tests (MSDA ops/test.py shapes, PrRoIPool test_prroi_pooling2d.py).
PrRoIPool has no CPU path in the reference, so the golden generator uses *this* restatement for
it: the score-head output is pinned only through the PrRoIPool KAT (documented in DESIGN.md).
"""
