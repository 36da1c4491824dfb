"""AdamW with global-norm gradient clipping on libmmt_hip.so (mmt_adamw_grad_norm / mmt_adamw_step).

Drop-in for the training step's `torch.nn.utils.clip_grad_norm_(params, max_norm)` followed by
`torch.optim.AdamW(param_groups, lr, weight_decay)` (train_script_mixformer.py:105-140,
ltr_trainer.py TRAIN.GRAD_CLIP_NORM, base_functions.py:362-400 parameter groups): three launches
over every parameter instead of PyTorch's per-group multi-tensor kernels, the norm, the clip and the
update.  The update pass also
  * zeroes the gradients in place (they stay allocated, so the device tables stay valid: zero_grad
    is then a no-op) -- or, with set_to_none=True, leaves them to zero_grad(set_to_none=True), which
    drops them so that autograd hands the next step's gradients over as .grad without an accumulate
    pass (only the small pointer table is rewritten when their addresses change), and
  * writes a bf16 shadow of the weights registered with `shadow=` (the backbone Linears): the next
    forward's GEMMs read it instead of casting each weight (mmt_amd.train._HipLinear), valid while
    the parameter's version counter is the one recorded with it.
Parameters without a gradient at a step are left untouched (as torch.optim does).
"""
import ctypes

import numpy as np
import torch

TENSOR_DTYPE = np.dtype([("p", "<u8"), ("g", "<u8"), ("m", "<u8"), ("v", "<u8"), ("shadow", "<u8"), ("n", "<i8"),
                         ("group", "<i4"), ("pad_", "<i4")])  # mmt_adamw_tensor
CHUNK_DTYPE = np.dtype([("tensor", "<i4"), ("pad_", "<i4"), ("offset", "<i8")])  # mmt_adamw_chunk
MAX_GROUPS = 8


class HipAdamW(torch.optim.Optimizer):
    """A torch.optim.Optimizer: `param_groups` are the live group dicts (the update reads each group's
    "lr" / "weight_decay" at every step, so the reference trainer's LR schedulers attach to it), and
    state_dict / load_state_dict carry exp_avg / exp_avg_sq and the step per parameter, as
    torch.optim.AdamW's do.  The bias corrections come from ONE device step counter (shared by every
    parameter, advanced once per step()); load_state_dict therefore requires one step value for all
    parameters (a state_dict written by torch.optim.AdamW over a run where every parameter had a
    gradient at every step has that)."""

    def __init__(self, param_groups, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2, shadow=(),
                 set_to_none=False):
        from ._lib import LIB
        self.lib = LIB
        self.set_to_none = set_to_none
        groups = []
        for g in param_groups:
            g = dict(g)
            g["params"] = [p for p in g["params"] if p.requires_grad]
            groups.append(g)
        if len(groups) > MAX_GROUPS:
            raise ValueError("at most %d parameter groups" % MAX_GROUPS)
        super().__init__(groups, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        self.betas, self.eps = betas, eps
        self.step_count = 0
        self.chunk = int(LIB.mmt_adamw_chunk_elems())
        shadow_ids = {id(p) for p in shadow}
        self._shadow = {}
        for g in self.groups:
            for p in g["params"]:
                if not (p.is_cuda and p.dtype == torch.float32 and p.is_contiguous()):
                    raise ValueError("HipAdamW takes contiguous fp32 device parameters")
                self.state[p] = {"exp_avg": torch.zeros_like(p), "exp_avg_sq": torch.zeros_like(p)}
                if id(p) in shadow_ids:
                    sh = p.detach().to(torch.bfloat16)
                    self._shadow[p] = sh
                    p._mmt_bf16 = (sh, p._version)
        self._key = None
        self.last_norm = None
        self.table_writes = 0

    @property
    def groups(self):
        """The live group dicts (load_state_dict replaces the list; schedulers write its "lr")."""
        return self.param_groups

    def _device_state(self, dev):
        if not hasattr(self, "_state"):
            self._state = torch.zeros(8, device=dev)  # norm, clip factor, bias corrections, step (int32)
        return self._state

    def state_dict(self):
        """torch.optim.AdamW's layout; every parameter's "step" is the device step counter."""
        step = float(self._state.view(torch.int32)[4].item()) if hasattr(self, "_state") else 0.0
        for p, st in self.state.items():
            st["step"] = torch.tensor(step)
        return super().state_dict()

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        steps = {float(st["step"]) for st in self.state.values() if "step" in st}
        if len(steps) > 1:
            raise ValueError("HipAdamW keeps one step counter for all parameters; the state_dict has %d "
                             "different per-parameter steps" % len(steps))
        dev = next(p for g in self.groups for p in g["params"]).device
        # Optimizer.load_state_dict keeps entries only for the parameters the saved state has: a
        # torch.optim.AdamW state_dict written before its first step, or one where a parameter never had a
        # gradient, leaves others without moments.  Those start from zero moments (what torch.optim.AdamW
        # would do at their first gradient); they share the device step counter for the bias corrections.
        for g in self.groups:
            for p in g["params"]:
                st = self.state[p]
                for k in ("exp_avg", "exp_avg_sq"):  # own contiguous fp32 copies on the parameter's device
                    # (Optimizer.load_state_dict keeps the source's tensors when device and dtype match:
                    # they are updated in place here)
                    st[k] = torch.empty_like(p).copy_(st[k]) if k in st else torch.zeros_like(p)
        self._device_state(dev).view(torch.int32)[4] = int(steps.pop()) if steps else 0
        self.step_count = int(self._state.view(torch.int32)[4].item())
        self._key = None  # the moment tensors are new: rebuild the device tables at the next step

    def zero_grad(self, set_to_none=False):
        """set_to_none: drop every gradient.  Else the update pass has zeroed the gradients it consumed
        (unless constructed with set_to_none=True); the others are cleared here."""
        for g in self.groups:
            for p in g["params"]:
                if p.grad is None:
                    continue
                if set_to_none:
                    p.grad = None
                elif self._key is None or self.set_to_none:
                    p.grad.zero_()

    def _tables(self, params):
        gkey = [p.grad.data_ptr() for _, p in params]
        pkey = [p.data_ptr() for _, p in params]
        if self._key is not None and gkey == self._key[1] and pkey == self._key[0]:
            return
        capturing = torch.cuda.is_current_stream_capturing()
        if capturing and (self._key is None or pkey != self._key[0]):
            raise RuntimeError("HipAdamW: the parameter set changed during hipGraph capture (run one eager step first)")
        for _, p in params:
            if not (p.grad.dtype == torch.float32 and p.grad.is_contiguous() and p.grad.shape == p.shape):
                raise ValueError("HipAdamW needs contiguous fp32 gradients of the parameter's shape")
        dev = params[0][1].device
        if self._key is None or pkey != self._key[0]:  # the parameter set: tensor rows and chunk list
            t = np.zeros(len(params), TENSOR_DTYPE)
            chunks = []
            for i, (gi, p) in enumerate(params):
                m, v = self.state[p]["exp_avg"], self.state[p]["exp_avg_sq"]
                sh = self._shadow.get(p)
                t[i] = (p.data_ptr(), 0, m.data_ptr(), v.data_ptr(), sh.data_ptr() if sh is not None else 0,
                        p.numel(), gi, 0)
                chunks += [(i, 0, o) for o in range(0, p.numel(), self.chunk)]
            self._tab = t
            self._chunks = torch.from_numpy(np.array(chunks, CHUNK_DTYPE).view(np.uint8).copy()).to(dev)
            self._nchunks = len(chunks)
            self._partial = torch.empty(self._nchunks, device=dev)
        self._tab["g"] = np.asarray(gkey, np.uint64)  # only the gradient addresses change between steps
        # through pinned memory, asynchronously: a pageable copy would hold the host until the stream drains.
        # Eager writes take a fresh pinned buffer (an earlier one may still be in flight) and reserve one
        # for a capture, because no pinned memory can be allocated while a stream captures.  Under hipGraph
        # capture (TrainStep.capture) the copy is recorded from that reserved buffer, which is then kept
        # alive and never rewritten: every replay reproduces the captured gradient addresses (the graph's
        # private memory pool), so the recorded table stays valid.
        data = self._tab.view(np.uint8)
        if capturing:
            host = getattr(self, "_cap_host", None)
            if host is None or host.numel() != data.size:
                raise RuntimeError("HipAdamW: no table buffer reserved for hipGraph capture (run one eager step first)")
            host.numpy()[:] = data
            self._captured_hosts = getattr(self, "_captured_hosts", []) + [host]
            self._cap_host = None
        else:
            host = torch.from_numpy(data.copy()).pin_memory()
            if getattr(self, "_cap_host", None) is None or self._cap_host.numel() != data.size:
                self._cap_host = torch.empty(data.size, dtype=torch.uint8).pin_memory()
        self._tens_host = host
        self._tens = host.to(dev, non_blocking=True)
        self.table_writes += 1
        self._device_state(dev)
        self._key = (pkey, gkey)

    @torch.no_grad()
    def step(self, max_norm=0.0):
        """clip_grad_norm_(max_norm) (skipped when max_norm <= 0) + one AdamW step: three launches with
        no host synchronisation and no host-side step state.  Capturable in a hipGraph after one eager
        step (TrainStep.capture): the pointer table write is recorded as a copy from a pinned buffer that
        stays valid because replays reuse the captured gradient addresses; the learning rates and weight
        decays are baked into the capture as kernel arguments (recapture after changing them).  The total
        gradient norm before clipping is `last_norm` (a device scalar) when max_norm > 0, else None (the
        norm pass is skipped)."""
        from ._lib import check
        params = [(gi, p) for gi, g in enumerate(self.groups) for p in g["params"] if p.grad is not None]
        if not params:
            return
        self._tables(params)
        self.step_count += 1
        n = len(self.groups)
        lr = (ctypes.c_float * n)(*[float(g["lr"]) for g in self.groups])
        wd = (ctypes.c_float * n)(*[float(g["weight_decay"]) for g in self.groups])
        check(self.lib.mmt_adamw_step(self._tens.data_ptr(), self._chunks.data_ptr(), self._nchunks,
                                      self._partial.data_ptr(), self._state.data_ptr(),
                                      ctypes.cast(lr, ctypes.c_void_p), ctypes.cast(wd, ctypes.c_void_p), n,
                                      float(self.betas[0]), float(self.betas[1]), float(self.eps), float(max_norm),
                                      0 if self.set_to_none else 1,
                                      torch.cuda.current_stream().cuda_stream), "mmt_adamw_step")
        self.last_norm = self._state[0] if max_norm > 0 else None
        for p in self._shadow:
            p._mmt_bf16 = (self._shadow[p], p._version)
