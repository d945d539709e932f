"""Drop-in for apex.optimizers.FusedAdam as the reference's train.py:146-152
uses it (FusedAdam(net_params, lr, eps=1e-15); weight decay 0, Adam mode,
bias correction on) on the native Adam kernel (ngp_adam_step: one launch per
parameter tensor, p / m / v updated in place).

A parameter of models.networks.NGP carries its fp16 shadow (the copy the
field kernels read); the same launch writes it, so the next forward finds it
current without a separate cast.  No CPU path: a parameter that is not a
contiguous fp32 CUDA tensor with a multiple of 4 elements raises, as apex's
CUDA-only optimizer would."""
import torch

import vren


class FusedAdam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, bias_correction=True, betas=(0.9, 0.999), eps=1e-8, adam_w_mode=True,
                 weight_decay=0.0, amsgrad=False):
        if amsgrad:
            raise RuntimeError("FusedAdam does not support the AMSGrad variant.")  # apex's message
        if weight_decay != 0.0 or not bias_correction:
            raise NotImplementedError("only the reference's configuration: weight_decay 0, bias correction on")
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        L = vren.lib()
        for group in self.param_groups:
            b1, b2 = group["betas"]
            for p in group["params"]:
                if p.grad is None:
                    continue
                g = p.grad
                if not (p.is_cuda and p.dtype == torch.float32 and p.is_contiguous() and g.is_contiguous()
                        and g.dtype == torch.float32 and p.numel() % 4 == 0):
                    raise RuntimeError("FusedAdam: parameters must be contiguous fp32 CUDA tensors with a multiple "
                                       "of 4 elements")
                st = self.state[p]
                if not st:
                    st["step"] = 0
                    st["exp_avg"] = torch.zeros_like(p)
                    st["exp_avg_sq"] = torch.zeros_like(p)
                st["step"] += 1
                shadow = getattr(p, "_ngp_shadow", None)
                if shadow is not None:
                    half = shadow.get()  # (allocated / current before the launch overwrites it)
                else:
                    half = st.get("half")
                    if half is None:
                        half = st["half"] = torch.empty(p.shape, dtype=torch.float16, device=p.device)
                vren._ok(L.ngp_adam_step(*[vren.c_void_p(t.data_ptr()) for t in
                                           (p, g, st["exp_avg"], st["exp_avg_sq"], half)],
                                         p.numel(), float(group["lr"]), float(b1), float(b2), float(group["eps"]),
                                         st["step"], 1.0, 0, vren._stream()), "FusedAdam")
                # the master changed in place under a raw pointer: bump its version so
                # autograd / other readers see the write, and mark the shadow current
                torch.autograd.graph.increment_version(p)
                if shadow is not None:
                    shadow.version = p._version
        return loss
