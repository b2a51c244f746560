"""Host-side checks of the flat parameter buffers (vst/reconet/_flat.py), no GPU needed."""
import pytest
import torch

from vst.reconet._flat import FlatParams, LossScaler


def test_parameters_are_views_of_the_flat_buffers():
    m = torch.nn.Sequential(torch.nn.Linear(4, 3), torch.nn.Linear(3, 2))
    flat = FlatParams(m)
    assert flat.numel == sum(p.numel() for p in m.parameters())
    for p in m.parameters():
        assert flat.p.data_ptr() <= p.data_ptr() < flat.p.data_ptr() + 4 * flat.numel
        assert flat.g.data_ptr() <= p.grad.data_ptr() < flat.g.data_ptr() + 4 * flat.numel


def test_update_invalidates_graphs_saved_before_it():
    """The Adam kernels update the parameters behind autograd's back; FlatParams bumps every
    parameter's own version counter (prm.data = view keeps it separate from the flat buffer's), so a
    graph that saved a parameter before the step refuses to run backward afterwards."""
    m = torch.nn.Linear(4, 3)
    flat = FlatParams(m)
    x = torch.randn(2, 4, requires_grad=True)
    y = (m(x) ** 2).sum()  # saves the weight for the input gradient
    flat._updated()
    with pytest.raises(RuntimeError, match="modified by an inplace operation"):
        y.backward()
    # a graph built after the update is fine
    (m(x) ** 2).sum().backward()


def test_loss_scaler_rejects_bad_settings():
    for kw in ({"init_scale": 0.0}, {"growth_factor": 0.5}, {"backoff_factor": 0.0}, {"backoff_factor": 2.0},
               {"growth_interval": 0}):
        with pytest.raises(ValueError):
            LossScaler("cpu", **kw)
    sc = LossScaler("cpu", init_scale=2.0 ** 12, step=5)
    assert sc.state_dict()["scale"] == 4096.0 and sc.state_dict()["step"] == 5
