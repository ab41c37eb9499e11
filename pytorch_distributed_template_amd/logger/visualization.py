"""TensorboardWriter (reference: ``/root/reference/logger/visualization.py:5-73``).

Same proxy API: ``set_step(step, mode)`` and ``add_*`` methods that append
``/<mode>`` to the tag and auto-log ``steps_per_sec`` at each ``set_step``.
It tries ``torch.utils.tensorboard`` then ``tensorboardX``; neither ships in
this image, so instead of silently dropping everything (reference
behaviour) scalars fall back to a ``scalars.jsonl`` file in the log dir.
"""
import importlib
import json
import time
from datetime import datetime
from pathlib import Path


class _JsonlScalarWriter:
    """Minimal SummaryWriter stand-in: one JSON line per scalar."""

    def __init__(self, log_dir):
        self._path = Path(log_dir) / "scalars.jsonl"
        self._fh = None

    def add_scalar(self, tag, value, step=None, *args, **kwargs):
        try:
            value = float(value)
        except Exception:  # tensors on device etc.
            value = float(value.item())
        if self._fh is None:
            self._fh = self._path.open("a")
        self._fh.write(json.dumps({"tag": tag, "value": value, "step": step, "time": time.time()}) + "\n")
        self._fh.flush()

    def add_scalars(self, main_tag, tag_scalar_dict, step=None, *args, **kwargs):
        for k, v in tag_scalar_dict.items():
            self.add_scalar(f"{main_tag}/{k}", v, step)


class TensorboardWriter:
    def __init__(self, log_dir, logger, enabled):
        self.writer = None
        self.selected_module = ""

        if enabled:
            log_dir = str(log_dir)
            for module in ("torch.utils.tensorboard", "tensorboardX"):
                try:
                    self.writer = importlib.import_module(module).SummaryWriter(log_dir)
                except ImportError:
                    continue
                self.selected_module = module  # the backend actually in use
                break

            if self.writer is None:
                logger.warning("Warning: visualization (Tensorboard) is configured to use, but neither "
                               "torch.utils.tensorboard nor tensorboardX is installed; scalars go to "
                               "scalars.jsonl in the run directory instead.")
                self.writer = _JsonlScalarWriter(log_dir)
                self.selected_module = "jsonl"

        self.step = 0
        self.mode = ""
        self.tb_writer_ftns = {
            "add_scalar", "add_scalars", "add_image", "add_images", "add_audio",
            "add_text", "add_histogram", "add_pr_curve", "add_embedding",
        }
        self.tag_mode_exceptions = {"add_histogram", "add_embedding"}
        self.timer = datetime.now()

    def set_step(self, step, mode="train"):
        self.mode = mode
        self.step = step
        if step == 0:
            self.timer = datetime.now()
        else:
            duration = datetime.now() - self.timer
            secs = duration.total_seconds()
            if secs > 0:
                self.add_scalar("steps_per_sec", 1 / secs)
            self.timer = datetime.now()

    def __getattr__(self, name):
        if name in self.tb_writer_ftns:
            add_data = getattr(self.writer, name, None)

            def wrapper(tag, data, *args, **kwargs):
                if add_data is not None:
                    if name not in self.tag_mode_exceptions:
                        tag = "{}/{}".format(tag, self.mode)
                    add_data(tag, data, self.step, *args, **kwargs)
            return wrapper
        raise AttributeError("type object '{}' has no attribute '{}'".format(self.selected_module, name))
