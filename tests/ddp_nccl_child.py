"""Child process of tests/test_gpu_ddp.py: the data-parallel training step over a REAL RCCL process group
(backend "nccl", one rank on cuda:0), against the single-process step on the same weights and batches.

Run as its own process (a fresh process group and a fresh HIP context; MASTER_ADDR / MASTER_PORT from the
parent).  Writes a JSON record to argv[1] and exits 0 when every check holds:
  1. eager, grad_compress="none": after 2 steps every gradient bitwise equal to the non-DDP step's, and the
     parameters after each AdamW step bitwise equal (at world 1 the average is x / 1 and the RCCL all-reduce
     a copy, so nothing may change); the head's BatchNorm2d modules are SyncBatchNorm (convert_sync_batchnorm,
     train_script_mixformer.py:105) in the DDP step;
  2. eager, grad_compress="bf16": every gradient within 2^-7 of its tensor's largest magnitude;
  3. the DDP step CAPTURED as one hipGraph (TrainStep.capture, the RCCL all-reduces recorded into it), two
     replays on the two batches: parameters bitwise equal to the captured non-DDP step's.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "multi-modal-tracking_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

B = int(os.environ.get("MMT_DDP_TEST_B", "2"))


def main(out_path):
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    from mmt_amd.model import build_mixformer_vit_rgbt, hot_path_cfg
    from mmt_amd.train import HipOps, TrainStep, synthetic_batch

    def net():
        torch.manual_seed(0)
        n = build_mixformer_vit_rgbt(hot_path_cfg(), train=False).cuda().train()
        # no RNG in the step (stochastic depth, dropout): the replicas are compared draw-free, eager and captured
        n.drop_path_rate = 0.0
        for m in n.modules():
            if isinstance(m, torch.nn.Dropout):
                m.p = 0.0
        return n

    g = torch.Generator().manual_seed(11)
    batches = [synthetic_batch(B, "cuda", g) for _ in range(2)]
    rec = {"backend": dist.get_backend(), "world": dist.get_world_size(), "B": B}

    def grads(n):
        return {k: p.grad.detach().clone() for k, p in n.named_parameters() if p.grad is not None}

    # 1 + 2: eager
    plain_net, ddp_net, bf_net = net(), net(), net()
    plain = TrainStep(plain_net, HipOps)
    ddp = TrainStep(ddp_net, HipOps, ddp=True, grad_compress="none")
    bf = TrainStep(bf_net, HipOps, ddp=True, grad_compress="bf16")
    rec["sync_bn_modules"] = sum(type(m) is torch.nn.SyncBatchNorm for m in ddp.net.modules())
    rec["buckets"] = len(ddp.reducer.buckets)
    worst_bf = 0.0
    for i in range(2):
        b = batches[i]
        lp = plain.backward(*b)["loss"].item()
        ld = ddp.backward(*b)["loss"].item()
        bf.backward(*b)
        gp, gd, gb = grads(plain_net), grads(ddp.net), grads(bf.net)
        assert set(gp) == set(gd) == set(gb), "gradient sets differ"
        neq = [k for k in gp if not torch.equal(gp[k], gd[k])]
        rec["step%d" % i] = {"loss_plain": lp, "loss_ddp": ld, "grads": len(gp), "grads_not_bitwise": neq[:8]}
        print(json.dumps(rec), flush=True)
        assert lp == ld, (lp, ld)
        assert not neq, neq[:8]
        for k in gp:
            sc = gp[k].abs().max().item() + 1e-20
            worst_bf = max(worst_bf, (gb[k] - gp[k]).abs().max().item() / sc)
        plain.apply()
        ddp.apply()
        bf.apply()
        pn = [k for (k, a), (_, c) in zip(plain_net.named_parameters(), ddp.net.named_parameters()) if not torch.equal(a, c)]
        assert not pn, pn[:8]
        # bf16 replica: the next step compares gradients at the plain replica's weights
        with torch.no_grad():
            for a, c in zip(plain_net.parameters(), bf.net.parameters()):
                c.copy_(a)
    rec["bf16_worst_rel_to_max"] = worst_bf
    assert worst_bf <= 2 ** -7, worst_bf
    del plain, ddp, bf, plain_net, ddp_net, bf_net
    torch.cuda.synchronize()
    torch.cuda.empty_cache()

    # 3: both steps captured, two replays each
    nets = [net(), net()]
    steps = [TrainStep(nets[0], HipOps), TrainStep(nets[1], HipOps, ddp=True, grad_compress="none")]
    static = [[[x.clone() for x in z] if isinstance(z, (list, tuple)) else z.clone() for z in batches[0]] for _ in steps]
    for st, sb in zip(steps, static):
        st.capture(*sb, warmup=1)
    losses = []
    for i in range(2):
        losses.append([float(st.replay(*batches[i % 2])["loss"]) for st in steps])
    torch.cuda.synchronize()
    pn = [k for (k, a), (_, c) in zip(nets[0].named_parameters(), steps[1].net.named_parameters()) if not torch.equal(a, c)]
    rec["captured"] = {"losses": losses, "params_not_bitwise": pn[:8]}
    assert all(a == b for a, b in losses), losses
    assert not pn, pn[:8]
    rec["ok"] = True
    with open(out_path, "w") as f:
        json.dump(rec, f)
    dist.destroy_process_group()


if __name__ == "__main__":
    try:
        main(sys.argv[1])
    except AssertionError as e:
        print("CHECK FAILED:", repr(e)[:2000], file=sys.stderr, flush=True)
        raise
