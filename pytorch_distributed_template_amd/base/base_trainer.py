"""BaseTrainer: epoch loop, monitor / early stop, checkpoint save & resume.

Reference: ``/root/reference/base/base_trainer.py:10-181``.

Kept identical (the public surface):
  * ``trainer`` config keys: ``epochs, save_dir, save_period, verbosity,
    monitor ("min val_loss" | "max <metric>" | "off"), early_stop, tensorboard``;
  * epoch summary lines ``'    {:15s}: {}'``;
  * checkpoint files ``checkpoint-epoch{N}.pth`` / ``model_best.pth`` with keys
    ``{arch, epoch, state_dict, optimizer, monitor_best, config}``
    (``state_dict`` without any DDP ``module.`` prefix).

Fixed: Q2 ``monitor: off`` no longer crashes (early_stop
defaults to inf); Q7 ``config`` is stored as a plain dict so checkpoints load
with ``torch.load(weights_only=True)``; Q17 ``arch`` is the unwrapped model
class; the LR-scheduler state is saved too (extra key ``lr_scheduler``) and
restored on resume; checkpoint writes are atomic (tmp + rename); the
early-stop vote is one broadcast from rank 0 instead of a pickled all-gather.
"""
from __future__ import annotations

import math
import os
from abc import abstractmethod

import torch

from ..logger import TensorboardWriter
from ..utils import dist as pdist


def unwrap_model(model):
    return model.module if hasattr(model, "module") and isinstance(model.module, torch.nn.Module) else model


class BaseTrainer:
    def __init__(self, model, criterion, metric_ftns, optimizer, config, lr_scheduler=None):
        self.config = config
        self.logger = config.get_logger("trainer", config["trainer"]["verbosity"])

        self.model = model
        self.criterion = criterion
        self.metric_ftns = metric_ftns
        self.optimizer = optimizer
        self.lr_scheduler = lr_scheduler

        cfg_trainer = config["trainer"]
        self.epochs = cfg_trainer["epochs"]
        self.save_period = cfg_trainer.get("save_period", 1)
        self.monitor = cfg_trainer.get("monitor", "off")
        self.early_stop = math.inf

        if self.monitor == "off":
            self.mnt_mode = "off"
            self.mnt_best = 0
        else:
            self.mnt_mode, self.mnt_metric = self.monitor.split()
            assert self.mnt_mode in ["min", "max"]
            self.mnt_best = math.inf if self.mnt_mode == "min" else -math.inf
            self.early_stop = cfg_trainer.get("early_stop", math.inf)
            if self.early_stop is None or self.early_stop <= 0:
                self.early_stop = math.inf

        self.start_epoch = 1
        self.checkpoint_dir = config.save_dir
        self.writer = TensorboardWriter(config.log_dir, self.logger,
                                        cfg_trainer.get("tensorboard", False) and pdist.is_main_process())

        if config.resume is not None:
            self._resume_checkpoint(config.resume)

    @abstractmethod
    def _train_epoch(self, epoch):
        raise NotImplementedError

    def _on_epoch_start(self, epoch):
        """Hook (e.g. ``sampler.set_epoch``)."""

    def train(self):
        not_improved_count = 0
        for epoch in range(self.start_epoch, self.epochs + 1):
            self._on_epoch_start(epoch)
            result = self._train_epoch(epoch)

            stop = False
            if pdist.is_main_process():
                log = {"epoch": epoch}
                log.update(result)
                for key, value in log.items():
                    self.logger.info("    {:15s}: {}".format(str(key), value))

                best = False
                if self.mnt_mode != "off":
                    try:
                        improved = (self.mnt_mode == "min" and log[self.mnt_metric] <= self.mnt_best) or \
                                   (self.mnt_mode == "max" and log[self.mnt_metric] >= self.mnt_best)
                    except KeyError:
                        self.logger.warning("Warning: Metric '{}' is not found. Model performance monitoring "
                                            "is disabled.".format(self.mnt_metric))
                        self.mnt_mode = "off"
                        improved = False
                    if improved:
                        self.mnt_best = log[self.mnt_metric]
                        not_improved_count = 0
                        best = True
                    else:
                        not_improved_count += 1

                if epoch % self.save_period == 0:
                    self._save_checkpoint(epoch, save_best=best)
                stop = not_improved_count > self.early_stop

            # early-stop consensus: every rank leaves the loop together
            stop = pdist.broadcast_object(stop, src=0)
            if stop:
                if pdist.is_main_process():
                    self.logger.info("Validation performance didn't improve for {} epochs. "
                                     "Training stops.".format(self.early_stop))
                break
        pdist.synchronize()

    # ------------------------------------------------------------------ checkpoint
    def _checkpoint_state(self, epoch):
        model = unwrap_model(self.model)
        state = {
            "arch": type(model).__name__,
            "epoch": epoch,
            "state_dict": {k: v for k, v in model.state_dict().items()},
            "optimizer": self.optimizer.state_dict(),
            "monitor_best": self.mnt_best,
            "config": self.config.to_dict(),
        }
        if self.lr_scheduler is not None:
            state["lr_scheduler"] = self.lr_scheduler.state_dict()
        return state

    @staticmethod
    def _atomic_save(state, path):
        tmp = str(path) + ".tmp"
        torch.save(state, tmp)
        os.replace(tmp, path)

    def _save_checkpoint(self, epoch, save_best=False):
        state = self._checkpoint_state(epoch)
        filename = str(self.checkpoint_dir / "checkpoint-epoch{}.pth".format(epoch))
        self._atomic_save(state, filename)
        self.logger.info("Saving checkpoint: {} ...".format(filename))
        if save_best:
            self._atomic_save(state, str(self.checkpoint_dir / "model_best.pth"))
            self.logger.info("Saving current best: model_best.pth ...")

    def _resume_checkpoint(self, resume_path):
        resume_path = str(resume_path)
        if pdist.is_main_process():
            self.logger.info("Loading checkpoint: {} ...".format(resume_path))
        checkpoint = load_checkpoint(resume_path)
        self.start_epoch = checkpoint["epoch"] + 1
        self.mnt_best = checkpoint["monitor_best"]

        if checkpoint["config"]["arch"] != self.config["arch"]:
            self.logger.warning("Warning: Architecture configuration given in config file is different from that "
                                "of checkpoint. This may yield an exception while state_dict is being loaded.")
        unwrap_model(self.model).load_state_dict(strip_module_prefix(checkpoint["state_dict"]))

        if checkpoint["config"]["optimizer"]["type"] != self.config["optimizer"]["type"]:
            self.logger.warning("Warning: Optimizer type given in config file is different from that of "
                                "checkpoint. Optimizer parameters not being resumed.")
        else:
            self.optimizer.load_state_dict(checkpoint["optimizer"])
            if self.lr_scheduler is not None and "lr_scheduler" in checkpoint:
                self.lr_scheduler.load_state_dict(checkpoint["lr_scheduler"])

        if pdist.is_main_process():
            self.logger.info("Checkpoint loaded. Resume training from epoch {}".format(self.start_epoch))

    # ------------------------------------------------------------------ collectives
    def reduce_loss(self, loss):
        return pdist.reduce_loss(loss)

    def _accumulate_predictions_from_multiple_gpus(self, predictions_per_gpu):
        """Gather a per-rank tensor (variable length) to rank 0; None elsewhere."""
        gathered = pdist.gather_tensors(predictions_per_gpu, dst=0)
        if gathered is None:
            return None
        return gathered


def strip_module_prefix(state_dict):
    """Remove a leading DDP ``module.`` prefix (only the leading one -- the
    reference replaced every occurrence of the substring)."""
    out = {}
    for k, v in state_dict.items():
        out[k[len("module."):] if k.startswith("module.") else k] = v
    return out


def load_checkpoint(path, map_location="cpu"):
    """Load a checkpoint written by this framework (plain tensors/dicts only)."""
    return torch.load(path, map_location=map_location, weights_only=True)
