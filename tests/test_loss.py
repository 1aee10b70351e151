"""Known-answer tests of the loss interface, restated from the reference's
tests/test_loss.py:6-108 (same inputs, same expected values and gradients)."""
import pytest
import torch

from drtvam_amd.loss import L2Loss, ThresholdedLoss


def T(vals, shape):
    return torch.tensor(vals, dtype=torch.float32).reshape(shape)


def grad_of(loss_fn, pred, target):
    pred = pred.clone().requires_grad_(True)
    loss = loss_fn(pred, target, 0 * target)
    loss.backward()
    return float(loss), pred.grad.reshape(-1)


def test_l2():
    target = T([1, 1, 0, 0], (2, 2, 1))
    loss, g = grad_of(L2Loss({'reduction': 'sum'}), T([1, 2, 3, 4], (2, 2, 1)), target)
    assert loss == 26
    assert torch.equal(g, torch.tensor([0., 2., 6., 8.]))

    loss, g = grad_of(L2Loss({'reduction': 'mean'}), T([1, 2, 3, 4], (2, 2, 1)), target)
    assert loss == 6.5
    assert torch.equal(g, torch.tensor([0., 0.5, 1.5, 2.]))

    target = T([0.2, 0.8, 0.5, 0.], (2, 2, 1))
    loss, g = grad_of(L2Loss({'reduction': 'sum'}), T([1., 1., 1., 1.], (2, 2, 1)), target)
    assert loss == pytest.approx(0.8 ** 2 + 0.2 ** 2 + 0.5 ** 2 + 1.)
    torch.testing.assert_close(g, torch.tensor([1.6, 0.4, 1., 2.]))

    # surface-aware target
    target = T([0.2, 0.8], (1, 1, 2))
    loss, g = grad_of(L2Loss({'reduction': 'sum'}), T([0.4, 0.3], (1, 1, 2)), target)
    assert loss == pytest.approx(0.2 * 0.6 ** 2 + 0.8 * 0.3 ** 2)
    torch.testing.assert_close(g, torch.tensor([-2 * 0.2 * 0.6, 2 * 0.8 * 0.3]))


@pytest.mark.parametrize("props,pred,loss_exp,grad_exp", [
    ({'K': 2, 'tl': 0.9, 'tu': 0.95, 'reduction': 'sum'}, [0.5, 0.97, 0.92, 0.5], 0.45 ** 2 + 0.02 ** 2,
     [-0.9, 0., 0.04, 0.]),
    ({'K': 2, 'tl': 0.9, 'tu': 0.95, 'reduction': 'mean'}, [0.5, 0.97, 0.92, 0.5], (0.45 ** 2 + 0.02 ** 2) / 4,
     [-0.225, 0., 0.01, 0.]),
    ({'K': 1, 'tl': 0.9, 'tu': 0.95, 'reduction': 'sum'}, [0.5, 1.1, 0.92, 0.5], 0.57, [-1, 1., 1., 0.]),
    ({'K': 2, 'tl': 0.4, 'tu': 0.95, 'reduction': 'sum'}, [0.5, 0.97, 0.92, 0.5], 0.45 ** 2 + 0.52 ** 2 + 0.1 ** 2,
     [-0.9, 0., 1.04, 0.2]),
    ({'K': 2, 'tl': 0.9, 'tu': 0.99, 'reduction': 'sum'}, [0.5, 0.97, 0.92, 0.5], 0.49 ** 2 + 0.02 ** 2 + 0.02 ** 2,
     [-0.98, -0.04, 0.04, 0.]),
])
def test_thresholded(props, pred, loss_exp, grad_exp):
    target = T([1, 1, 0, 0], (2, 2))
    loss, g = grad_of(ThresholdedLoss(props), T(pred, (2, 2, 1)), target)
    assert loss == pytest.approx(loss_exp, rel=1e-5)
    torch.testing.assert_close(g, torch.tensor(grad_exp, dtype=torch.float32), rtol=1e-5, atol=1e-6)


def test_thresholded_surface_aware():
    lf = ThresholdedLoss({'K': 2, 'tl': 0.9, 'tu': 0.95, 'reduction': 'sum'})
    target = T([0.2, 0.8, 2, 2], (2, 1, 2))
    loss, g = grad_of(lf, T([0.2, 0.1, 0.96, 0.92], (2, 1, 2)), target)
    assert loss == pytest.approx(0.2 * 0.75 ** 2 + 0.5 * 0.02 ** 2, rel=1e-5)
    torch.testing.assert_close(g, torch.tensor([-2 * 0.2 * 0.75, 0., 0., 2 * 0.5 * 0.02]), rtol=1e-5, atol=1e-6)


def test_threshold_validation():
    with pytest.raises(ValueError):
        ThresholdedLoss({'tl': 0.95, 'tu': 0.9})
    with pytest.raises(ValueError):
        ThresholdedLoss({'reduction': 'max'})


def test_registries():
    import drtvam_amd
    from drtvam_amd import loss as L
    assert set(L.losses) == {'l2', 'threshold'}
    with pytest.raises(ValueError):
        drtvam_amd.register_loss('l2', L.L2Loss)

    class MyLoss(L.Loss):
        pass
    drtvam_amd.register_loss('mine', MyLoss)
    assert L.losses['mine'] is MyLoss
    del L.losses['mine']
