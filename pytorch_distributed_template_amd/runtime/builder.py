"""Builds every training/eval component from a ConfigParser.

Shared by ``train.py``, ``test.py`` and the tests so that the wiring in the
reference's ``train.py:16-74`` / ``test.py:14-101`` lives in one place.
Registries (``init_obj`` lookups, searched in order):
  arch        -> pytorch_distributed_template_amd.models
  loaders     -> pytorch_distributed_template_amd.data
  loss        -> pytorch_distributed_template_amd.models.loss
  metrics     -> pytorch_distributed_template_amd.models.metric
  optimizer   -> pytorch_distributed_template_amd.optim, then torch.optim (SGD / Adam /
                 AdamW become the fused HIP optimizers on the native GPU path)
  lr_scheduler-> torch.optim.lr_scheduler (optional: null / missing disables it)

Extra (optional) ``trainer`` keys, all defaulting to reference behaviour:
  precision "fp32"|"bf16", channels_last bool, backend "auto"|"native"|"torch",
  ddp {bucket_cap_mb, broadcast_buffers, gradient_as_bucket_view, comm_hook},
  len_epoch int (iteration-based epochs), log_images bool, fused_optimizer bool,
  hip_graph bool (capture the training step -- DDP all-reduce included -- as one HIP
  graph after a warm-up and replay it; needs a fused optimizer, built capturable).
"""
from __future__ import annotations

import torch

from .. import data as module_data
from .. import models as module_arch
from .. import optim as module_optim
from ..models import loss as module_loss
from ..models import metric as module_metric
from ..ops import fused
from ..parallel import pretune_for_ddp, wrap_ddp


def build_model(config, device):
    model = config.init_obj("arch", module_arch)
    tcfg = config["trainer"]
    if tcfg.get("backend"):
        fused.set_backend(tcfg["backend"])
    model = model.to(device)
    if tcfg.get("channels_last", False):
        model = model.to(memory_format=torch.channels_last)
    return model


def build_criterion_metrics(config):
    criterion = getattr(module_loss, config["loss"])
    metrics = [getattr(module_metric, met) for met in config["metrics"]]
    return criterion, metrics


# torch.optim names a config may use -> the multi-tensor HIP optimizer with the same
# semantics and interchangeable state_dict (optim/fused.py), and the args it accepts
_FUSED_FOR = {
    "SGD": ("FusedSGD", {"lr", "momentum", "dampening", "weight_decay", "nesterov"}),
    "Adam": ("FusedAdam", {"lr", "betas", "eps", "weight_decay", "amsgrad"}),
    "AdamW": ("FusedAdamW", {"lr", "betas", "eps", "weight_decay", "amsgrad"}),
}


def build_optimizer(config, model):
    """``optimizer.type`` is looked up in ``optim`` first, then ``torch.optim``. On the
    native GPU path a torch.optim SGD / Adam / AdamW (e.g. the reference's ``"Adam"``)
    becomes its fused HIP counterpart -- one launch per step instead of torch's foreach
    kernels -- unless ``trainer.fused_optimizer`` is false."""
    params = [p for p in model.parameters() if p.requires_grad]
    ocfg = config["optimizer"]
    fused_name, allowed = _FUSED_FOR.get(ocfg["type"], (None, None))
    if (fused_name and config["trainer"].get("fused_optimizer", True) and params
            and set(ocfg.get("args", {})) <= allowed and fused.use_native(params[0])):
        # fp32-only models (LeNet) read no bf16 weight shadow
        optimizer = getattr(module_optim, fused_name)(params, **dict(ocfg.get("args", {})),
                                                      write_bf16_shadow=config["trainer"].get("precision") == "bf16",
                                                      capturable=bool(config["trainer"].get("hip_graph", False)))
    else:
        extra = {}
        if config["trainer"].get("hip_graph", False) and str(ocfg["type"]).startswith("Fused") \
                and "capturable" not in ocfg.get("args", {}):
            extra["capturable"] = True  # (optim.Fused*: lr / step counts in device memory)
        optimizer = config.init_obj("optimizer", [module_optim, torch.optim], params, **extra)
    lr_scheduler = None
    if config.get("lr_scheduler"):
        lr_scheduler = config.init_obj("lr_scheduler", torch.optim.lr_scheduler, optimizer)
    return optimizer, lr_scheduler


def wrap_model(config, model, device):
    ddp_cfg = dict(config["trainer"].get("ddp", {}))

    def wrap():
        return wrap_ddp(model, device,
                        bucket_cap_mb=ddp_cfg.get("bucket_cap_mb", 64),
                        broadcast_buffers=ddp_cfg.get("broadcast_buffers", True),
                        gradient_as_bucket_view=ddp_cfg.get("gradient_as_bucket_view", True),
                        comm_hook=ddp_cfg.get("comm_hook"),
                        find_unused_parameters=ddp_cfg.get("find_unused_parameters", False))

    if config["trainer"].get("hip_graph", False) and device.type == "cuda":
        # PyTorch's whole-network DDP capture recipe: the reducer is built on a side stream
        # (the Trainer runs its warm-up steps and the capture on that stream too)
        side = torch.cuda.Stream(device=device)
        side.wait_stream(torch.cuda.current_stream(device))
        with torch.cuda.stream(side):
            model = wrap()
        torch.cuda.current_stream(device).wait_stream(side)
        # the Trainer runs the warm-up and the capture on THIS stream: DDP binds its gradient
        # accumulators to the construction stream (another stream: NaN gradients after capture)
        model._pdt_capture_stream = side
        return model
    return wrap()


def pretune_model(config, model, data_loader, criterion, device):
    """World size > 1 on the native backend: one forward+backward on rank 0 tunes
    the kernel variants, which are broadcast to every rank before DDP wraps the
    model (``parallel.pretune_for_ddp``). Other cases: no-op."""
    from ..utils.dist import get_world_size
    if get_world_size() <= 1 or device.type != "cuda":
        return

    def step():
        data, target = next(iter(data_loader))
        data, target = data.to(device, non_blocking=True), target.to(device, non_blocking=True)
        if config["trainer"].get("channels_last", False) and data.dim() == 4 \
                and getattr(data, "pdt_nhwc_pad", None) is None:
            data = data.contiguous(memory_format=torch.channels_last)
        with torch.autocast(device_type=device.type, dtype=autocast_dtype(config, device) or torch.bfloat16,
                            enabled=autocast_dtype(config, device) is not None):
            loss = criterion(model(data), target)
        loss.backward()

    pretune_for_ddp(model, step)


def autocast_dtype(config, device):
    """bf16 precision: native kernels are bf16 already (no autocast); the torch
    path uses autocast(bf16) -- the reference-equivalent mixed precision."""
    if config["trainer"].get("precision", "fp32") != "bf16":
        return None
    if device.type == "cuda" and fused.get_backend() != "torch":
        from ..ops import native_ops
        if native_ops.available():
            return None
    return torch.bfloat16


def build_loader(config, name):
    return config.init_obj(name, module_data)
