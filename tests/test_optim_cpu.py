import pytest
import torch

from pytorch_distributed_template_amd.optim import FusedAdam, FusedAdamW, FusedSGD


@pytest.mark.parametrize("kind", ["sgd", "nesterov", "adam", "adam_ams", "adamw"])
def test_cpu_fallback_matches_torch(kind):
    torch.manual_seed(0)
    ps = [torch.randn(5, 3, requires_grad=True), torch.randn(7, requires_grad=True)]
    qs = [p.detach().clone().requires_grad_(True) for p in ps]
    mk = {
        "sgd": (lambda x: FusedSGD(x, lr=0.1, momentum=0.9, weight_decay=1e-3),
                lambda x: torch.optim.SGD(x, lr=0.1, momentum=0.9, weight_decay=1e-3)),
        "nesterov": (lambda x: FusedSGD(x, lr=0.1, momentum=0.9, nesterov=True),
                     lambda x: torch.optim.SGD(x, lr=0.1, momentum=0.9, nesterov=True)),
        "adam": (lambda x: FusedAdam(x, lr=1e-2, weight_decay=1e-2), lambda x: torch.optim.Adam(x, lr=1e-2,
                                                                                              weight_decay=1e-2)),
        "adam_ams": (lambda x: FusedAdam(x, lr=1e-2, amsgrad=True), lambda x: torch.optim.Adam(x, lr=1e-2,
                                                                                             amsgrad=True)),
        "adamw": (lambda x: FusedAdamW(x, lr=1e-2), lambda x: torch.optim.AdamW(x, lr=1e-2)),
    }[kind]
    a, b = mk[0](ps), mk[1](qs)
    for _ in range(5):
        for p, q in zip(ps, qs):
            g = torch.randn_like(p)
            p.grad, q.grad = g.clone(), g.clone()
        a.step()
        b.step()
    for p, q in zip(ps, qs):
        assert torch.allclose(p, q, atol=1e-6), (p - q).abs().max()
    sd = a.state_dict()
    b.load_state_dict(sd)


class _Cfg(dict):
    """The two ConfigParser calls build_optimizer makes: cfg[key] and init_obj."""

    def init_obj(self, name, module, *args):
        spec = self[name]
        for m in (module if isinstance(module, (list, tuple)) else [module]):
            if hasattr(m, spec["type"]):
                return getattr(m, spec["type"])(*args, **spec["args"])
        raise AttributeError(spec["type"])


def _mnist_opt_cfg(**trainer):
    return _Cfg(optimizer={"type": "Adam", "args": {"lr": 1e-3, "weight_decay": 0, "amsgrad": True}},
                trainer=dict(trainer))


def test_build_optimizer_keeps_torch_adam_on_cpu():
    from pytorch_distributed_template_amd.runtime.builder import build_optimizer
    opt, sched = build_optimizer(_mnist_opt_cfg(), torch.nn.Linear(4, 3))
    assert type(opt) is torch.optim.Adam and sched is None
