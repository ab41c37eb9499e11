#!/usr/bin/env python
"""Evaluation entry point -- same CLI as the reference ``/root/reference/test.py:104-128``.

    python test.py -r path/to/checkpoint-epochN.pth [-c override.json] [-s save_dir] [--seed N]

Loads the checkpoint (``torch.load(weights_only=True)``: our checkpoints hold
only tensors and plain dicts), runs distributed inference over
``test_loader`` with unpadded per-rank shards, gathers logits/targets to
rank 0 as fixed-shape tensors and logs
``{'loss': sum(loss*bs)/len(dataset), <metric>: ...}`` like the reference.
Fixes ``--seed`` (the reference hit a NameError).
"""
import argparse

import torch

from pytorch_distributed_template_amd.base.base_trainer import load_checkpoint, strip_module_prefix
from pytorch_distributed_template_amd.config import ConfigParser
from pytorch_distributed_template_amd.runtime import (autocast_dtype, build_criterion_metrics, build_loader,
                                                      build_model)
from pytorch_distributed_template_amd.utils import dist as pdist
from pytorch_distributed_template_amd.utils.util import seed_everything, set_deterministic


@torch.no_grad()
def main(args, config, device):
    logger = config.get_logger("test")
    model = build_model(config, device)
    data_loader = build_loader(config, "test_loader")
    loss_fn, metric_fns = build_criterion_metrics(config)

    if pdist.is_main_process():
        logger.info(model)
        logger.info("Loading checkpoint: {} ...".format(config.resume))
    checkpoint = load_checkpoint(config.resume, map_location=device)
    model.load_state_dict(strip_module_prefix(checkpoint["state_dict"]))
    model.eval()

    ac = autocast_dtype(config, device)
    channels_last = config["trainer"].get("channels_last", False)
    total_loss = torch.zeros((), dtype=torch.float64, device=device)
    outputs, targets = [], []
    for data, target in data_loader:
        data, target = data.to(device, non_blocking=True), target.to(device, non_blocking=True)
        # a loader's NHWC-padded batch (``pdt_nhwc_pad``) is already in the layout the native
        # stem reads in place: re-laying it out would copy it and drop the tag (as in Trainer)
        if channels_last and data.dim() == 4 and getattr(data, "pdt_nhwc_pad", None) is None:
            data = data.contiguous(memory_format=torch.channels_last)
        with torch.autocast(device_type=device.type, dtype=ac or torch.float32, enabled=ac is not None):
            output = model(data)
            loss = loss_fn(output, target)
        outputs.append(output.float())
        targets.append(target)
        total_loss += loss.double() * data.shape[0]

    out = torch.cat(outputs) if outputs else torch.zeros((0, 1), device=device)
    tgt = torch.cat(targets) if targets else torch.zeros((0,), dtype=torch.long, device=device)
    if pdist.get_world_size() > 1:
        torch.distributed.all_reduce(total_loss)
    outs = pdist.gather_tensors(out, dst=0)
    tgts = pdist.gather_tensors(tgt, dst=0)
    log = {"loss": float(total_loss.item()) / len(data_loader.dataset)}
    if pdist.is_main_process():
        out_all, tgt_all = torch.cat(outs), torch.cat(tgts)
        log.update({met.__name__: met(out_all, tgt_all) for met in metric_fns})
        logger.info(log)
    return log


def cli(argv=None):
    args = argparse.ArgumentParser(description="MI355X distributed training template (evaluation)")
    args.add_argument("-c", "--config", default=None, type=str, help="config file path (default: None)")
    args.add_argument("-r", "--resume", default=None, type=str, help="path to checkpoint")
    args.add_argument("-l", "--local_rank", "--local-rank", dest="local_rank", default=None, type=int)
    args.add_argument("-s", "--save_dir", default=None, type=str, help="dir of save path")
    args.add_argument("--seed", type=int, default=None, help="Random seed.")
    args.add_argument("--deterministic", action="store_true")
    args.add_argument("--backend", default=None, choices=["auto", "native", "torch"])
    ns = args.parse_args(argv)
    assert ns.resume is not None, "Testing mode requires model path!"
    device = pdist.init_distributed(ns.local_rank)
    ns, config = ConfigParser.from_args(ns, training=False)
    if ns.backend:
        config["trainer"]["backend"] = ns.backend
    if ns.seed is not None:
        seed_everything(ns.seed, ns.deterministic)
    elif ns.deterministic:
        set_deterministic(True)
    try:
        return main(ns, config, device)
    finally:
        pdist.cleanup()


if __name__ == "__main__":
    cli()
