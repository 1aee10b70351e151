"""Loss functions (mirror of drtvam/loss.py) on torch tensors.

``loss_fn(x, target, patterns) -> scalar`` keeps the reference contract
(loss.py:28-59): ``x`` is the dose [Z, Y, X, C]; ``target`` is broadcast
from [Z, Y, X] / [Z, Y, X, 1] (binary or greyscale) or is a 2-channel
surface-aware volume; the sparsity term over ``patterns`` is reduced
separately.  Gradients come from torch autograd.

``ThresholdedLoss.fused_value`` / ``fused_value_grad`` evaluate the binary-
target case with one HIP kernel pass (value + dL/dx), which is what the
optimizer uses on the GPU for the main evaluation and the Armijo probes of
lbfgs.py:256-266 (x = vol + alpha * dvol, never materialised).
"""
from __future__ import annotations

import torch


def relu(x):
    return torch.where(x > 0, x, torch.zeros((), dtype=x.dtype, device=x.device))


def _sum(x):
    return torch.sum(x)


def _mean(x):
    return torch.mean(x)


class Loss:
    def __init__(self, props):
        reduction = props.get('reduction', 'sum')
        if reduction == 'sum':
            self.reduction = _sum
        elif reduction == 'mean':
            self.reduction = _mean
        else:
            raise ValueError(f"Invalid reduction method: '{reduction}'.")
        self.reduction_name = reduction

    def eval_in(self, x):
        raise NotImplementedError

    def eval_out(self, x):
        raise NotImplementedError

    def eval(self, x, target, patterns):
        raise NotImplementedError

    def eval_sparsity(self, patterns):
        raise NotImplementedError

    def __call__(self, x, target, patterns):
        if tuple(x.shape) != tuple(target.shape):
            if len(x.shape) == len(target.shape) + 1 and x.shape[-1] == 1:
                target = target[..., None]
            else:
                raise ValueError(f"Input and target shapes do not match: {tuple(x.shape)} != {tuple(target.shape)}")

        if target.shape[-1] == 1:
            loss, loss_patterns = self.eval(x, target, patterns)
        elif target.shape[-1] == 2:
            w_in = target[..., 0] / (target[..., 0] + target[..., 1])
            w_out = target[..., 1] / (target[..., 0] + target[..., 1])
            loss = w_in * self.eval_in(x[..., 0]) + w_out * self.eval_out(x[..., 1])
            loss_patterns = self.eval_sparsity(patterns)
        else:
            raise ValueError(f"[Loss] Received tensors of invalid shape: {tuple(target.shape)}. "
                             "The last dimension should be either 1 or 2.")
        return self.reduction(loss) + self.reduction(loss_patterns)


class L2Loss(Loss):
    def __init__(self, props):
        super().__init__(props)
        self.M = props.get('M', 4)
        self.weight_sparsity = props.get('weight_sparsity', 0)

    def eval_in(self, x):
        return torch.square(x - 1.)

    def eval_out(self, x):
        return torch.square(x)

    def eval(self, x, target, patterns):
        return torch.square(x - target), 0 * patterns

    def eval_sparsity(self, patterns):
        return patterns ** self.M * self.weight_sparsity


class ThresholdedLoss(Loss):
    """Thresholded loss (Wechsler et al. 2024), loss.py:82-132."""

    def __init__(self, props):
        super().__init__(props)
        self.K = props.get('K', 2)
        self.M = props.get('M', 4)
        self.tl = props.get('tl', 0.9)
        self.tu = props.get('tu', 0.95)
        self.weight_object = props.get('weight_object', 1)
        self.weight_void = props.get('weight_void', 1)
        self.weight_limit = props.get('weight_limit', 1)
        self.weight_sparsity = props.get('weight_sparsity', 0)
        if self.tl >= self.tu:
            raise ValueError(f"[ThresholdedLoss] Lower threshold ({self.tl}) must be smaller than upper threshold ({self.tu})")

    def eval_in(self, x):
        return self.weight_object * relu(self.tu - x) ** self.K + self.weight_limit * relu(x - 1.) ** self.K

    def eval_out(self, x):
        return self.weight_void * relu(x - self.tl) ** self.K

    def eval_sparsity(self, patterns):
        return torch.abs(patterns) ** self.M * self.weight_sparsity

    def eval(self, x, target, patterns):
        return torch.where(target > 0, self.eval_in(x), self.eval_out(x)), self.eval_sparsity(patterns)

    # ---- fused HIP path (binary / greyscale target, integer K) -------------
    def fusable(self, x, target) -> bool:
        return (x.is_cuda and float(self.K).is_integer() and 1 <= int(self.K) <= 16 and x.dtype == torch.float32
                and target.dtype == torch.float32 and target.numel() == x.numel())

    def _sparsity_value(self, patterns):
        if not self.weight_sparsity or patterns is None:
            return None
        p = patterns.detach()
        return self.reduction(torch.abs(p) ** self.M * self.weight_sparsity).to(torch.float64)

    def _target_mask(self, target):
        """(bit mask, bit offset) of target's object test (engine.target_mask), built once per target:
        the mask covers the contiguous base tensor a view (a slab of the film) comes from, and is
        rebuilt when that tensor is written in place (its version counter moves).  None: use the f32
        target."""
        base = target if target._base is None else target._base
        if not (base.is_contiguous() and base.dtype == torch.float32 and base.is_cuda):
            return None
        key = (base.data_ptr(), base.numel(), base._version)
        c = getattr(self, '_mask_cache', None)
        if c is None or c[0] != key:
            from .engine import target_mask
            c = (key, base, target_mask(base))
            self._mask_cache = c
        return c[2], (target.data_ptr() - base.data_ptr()) // 4

    def fused_value(self, x, target, patterns, dx=None, alpha=0.0, count=None):
        """Loss of x (+ alpha*dx) as an f64 device scalar, one kernel pass.  ``patterns=None``
        leaves out the sparsity term; ``count`` is the element count of a 'mean' reduction
        when x is one slab of the film."""
        from .engine import loss_threshold
        scale = 1.0 / (count or x.numel()) if self.reduction_name == 'mean' else 1.0
        m = self._target_mask(target)
        v = loss_threshold(x.reshape(-1), target.reshape(-1), int(self.K), self.tl, self.tu, self.weight_object,
                           self.weight_void, self.weight_limit, scale,
                           None if dx is None else dx.reshape(-1), alpha, mask=m[0] if m else None,
                           mask_bit0=m[1] if m else 0)
        s = self._sparsity_value(patterns)
        return v if s is None else v + s

    def fused_values(self, x, target, patterns, dx, alphas, count=None):
        """Losses of x + a*dx for every a in alphas (<= 8) as an f64 device vector, one kernel
        pass (the Armijo probes of the line search; ``patterns`` / ``count`` as in fused_value)."""
        from .engine import loss_threshold_probes
        scale = 1.0 / (count or x.numel()) if self.reduction_name == 'mean' else 1.0
        m = self._target_mask(target)
        v = loss_threshold_probes(x.reshape(-1), dx.reshape(-1), alphas, target.reshape(-1), int(self.K), self.tl,
                                  self.tu, self.weight_object, self.weight_void, self.weight_limit, scale,
                                  mask=m[0] if m else None, mask_bit0=m[1] if m else 0)
        s = self._sparsity_value(patterns)
        return v if s is None else v + s

    def fused_value_grad(self, x, target, patterns, grad_out, count=None):
        """Loss value (f64 device scalar) and dL/dx written into grad_out, one kernel pass
        (``patterns`` / ``count`` as in fused_value)."""
        from .engine import loss_threshold
        scale = 1.0 / (count or x.numel()) if self.reduction_name == 'mean' else 1.0
        m = self._target_mask(target)
        v = loss_threshold(x.reshape(-1), target.reshape(-1), int(self.K), self.tl, self.tu, self.weight_object,
                           self.weight_void, self.weight_limit, scale, grad=grad_out.reshape(-1),
                           mask=m[0] if m else None, mask_bit0=m[1] if m else 0)
        s = self._sparsity_value(patterns)
        return v if s is None else v + s

    def sparsity_grad(self, patterns):
        """d/dp of the sparsity term (added to the adjoint gradient)."""
        if not self.weight_sparsity:
            return None
        p = patterns.detach()
        g = self.weight_sparsity * self.M * torch.abs(p) ** (self.M - 1) * torch.sign(p)
        if self.reduction_name == 'mean':
            g = g / p.numel()
        return g


losses = {
    'l2': L2Loss,
    'threshold': ThresholdedLoss,
}
