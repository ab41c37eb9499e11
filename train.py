#!/usr/bin/env python
"""Training entry point -- same CLI as the reference ``/root/reference/train.py:77-108``.

    python train.py -c config/config.json [-r ckpt] [-s save_dir] [--no-validate]
                    [--seed N] [--deterministic] [--lr F] [--bs N]
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 train.py -c config/resnet50_bf16.json

Differences: the process group is initialised *before* the
config/run dir so all ranks agree on ONE run dir (Q5); ``--local-rank``,
``--local_rank`` and ``LOCAL_RANK`` are all accepted (Q4/Q16); ``--bs`` targets
``train_loader;args;batch_size`` (Q3); backend is RCCL on GPU and gloo on CPU.
"""
import argparse
import collections

import torch

from pytorch_distributed_template_amd.config import ConfigParser
from pytorch_distributed_template_amd.runtime import (autocast_dtype, build_criterion_metrics, build_loader,
                                                      build_model, build_optimizer, pretune_model,
                                                      wrap_model)
from pytorch_distributed_template_amd.trainer import Trainer
from pytorch_distributed_template_amd.utils import dist as pdist
from pytorch_distributed_template_amd.utils.util import seed_everything, set_deterministic


def main(args, config, device):
    logger = config.get_logger("train")

    model = build_model(config, device)
    criterion, metrics = build_criterion_metrics(config)
    optimizer, lr_scheduler = build_optimizer(config, model)

    data_loader = build_loader(config, "train_loader")
    valid_data_loader = None if args.no_validate else build_loader(config, "valid_loader")
    tcfg = config["trainer"]
    pretune_model(config, model, data_loader, criterion, device)  # N ranks agree on kernel variants
    model = wrap_model(config, model, device)

    if pdist.is_main_process():
        if pdist.is_dist_ready():
            logger.info("process group: {}, world size {}".format(torch.distributed.get_backend(),
                                                                   pdist.get_world_size()))
        logger.info(model)

    trainer = Trainer(model, criterion, metrics, optimizer, config=config, device=device,
                      data_loader=data_loader, valid_data_loader=valid_data_loader, lr_scheduler=lr_scheduler,
                      len_epoch=tcfg.get("len_epoch"), autocast_dtype=autocast_dtype(config, device),
                      channels_last=tcfg.get("channels_last", False))
    trainer.train()
    return trainer


def build_argparser():
    args = argparse.ArgumentParser(description="MI355X distributed training template")
    args.add_argument("-c", "--config", default=None, type=str, help="config file path (default: None)")
    args.add_argument("-r", "--resume", default=None, type=str, help="path to latest checkpoint (default: None)")
    args.add_argument("-l", "--local_rank", "--local-rank", dest="local_rank", default=None, type=int,
                      help="local rank of gpu (LOCAL_RANK env wins)")
    args.add_argument("-s", "--save_dir", default=None, type=str, help="dir of save path")
    args.add_argument("--no-validate", action="store_true",
                      help="Whether not to evaluate the checkpoint during training.")
    args.add_argument("--seed", type=int, default=None, help="Random seed.")
    args.add_argument("--deterministic", action="store_true",
                      help="Deterministic kernels (MIOpen / torch) when --seed is given.")
    args.add_argument("--backend", default=None, choices=["auto", "native", "torch"],
                      help="kernel backend override (default: config trainer.backend or auto)")
    return args


CustomArgs = collections.namedtuple("CustomArgs", "flags type target")
OPTIONS = [
    CustomArgs(["--lr", "--learning_rate"], type=float, target="optimizer;args;lr"),
    CustomArgs(["--bs", "--batch_size"], type=int, target="train_loader;args;batch_size"),
    CustomArgs(["--epochs"], type=int, target="trainer;epochs"),
]


def cli(argv=None):
    parser = build_argparser()
    for opt in OPTIONS:
        parser.add_argument(*opt.flags, default=None, type=opt.type)
    ns = parser.parse_args(argv)
    device = pdist.init_distributed(ns.local_rank)
    ns, config = ConfigParser.from_args(ns, OPTIONS, training=True)
    if ns.backend:
        config["trainer"]["backend"] = ns.backend
    if ns.seed is not None:
        seed_everything(ns.seed, ns.deterministic)
    else:
        set_deterministic(ns.deterministic)
    try:
        return main(ns, config, device)
    finally:
        pdist.cleanup()


if __name__ == "__main__":
    cli()
