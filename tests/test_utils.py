import json
import logging

import torch

from pytorch_distributed_template_amd.logger import TensorboardWriter
from pytorch_distributed_template_amd.utils import MetricTracker, inf_loop, read_json, write_json
from pytorch_distributed_template_amd.utils.image import make_grid


def test_metric_tracker_numbers_and_tensors():
    mt = MetricTracker("loss", "acc")
    mt.update("loss", 1.0)
    mt.update("loss", torch.tensor(3.0))
    mt.update("acc", 0.5, n=4)
    mt.update("acc", 1.0, n=4)
    r = mt.result()
    assert r["loss"] == 2.0 and r["acc"] == 0.75
    mt.reset()
    assert mt.avg("loss") == 0.0


def test_json_roundtrip_ordered(tmp_path):
    d = {"b": 1, "a": [1, 2]}
    write_json(d, tmp_path / "x.json")
    r = read_json(tmp_path / "x.json")
    assert list(r.keys()) == ["b", "a"]


def test_inf_loop():
    it = inf_loop([1, 2])
    assert [next(it) for _ in range(5)] == [1, 2, 1, 2, 1]


def test_make_grid_shapes():
    g = make_grid(torch.rand(10, 1, 28, 28), nrow=8, normalize=True)
    assert g.shape == (3, 2 * 30 + 2, 8 * 30 + 2)


def test_tensorboard_writer_fallback_jsonl(tmp_path):
    w = TensorboardWriter(tmp_path, logging.getLogger("t"), True)
    w.set_step(0)
    w.add_scalar("loss", 1.5)
    w.set_step(1, "valid")
    w.add_scalar("acc", torch.tensor(0.25))
    if w.selected_module == "jsonl":
        lines = [json.loads(l) for l in (tmp_path / "scalars.jsonl").read_text().splitlines()]
        tags = [l["tag"] for l in lines]
        assert "loss/train" in tags and "acc/valid" in tags and "steps_per_sec/valid" in tags
    off = TensorboardWriter(tmp_path, logging.getLogger("t"), False)
    off.add_scalar("x", 1.0)  # no-op


def test_shipped_logger_config_json_is_the_default(tmp_path):
    """logger/logger_config.json ships with the reference schema (/root/reference/logger/logger.py:7)
    and setup_logging reads it by default: console + rotating info.log in the run dir."""
    import json
    import logging
    from pytorch_distributed_template_amd.logger.logger import (DEFAULT_LOG_CONFIG, default_log_config,
                                                                setup_logging)
    cfg = json.loads(DEFAULT_LOG_CONFIG.read_text())
    assert cfg == default_log_config()
    assert cfg["handlers"]["info_file_handler"]["class"] == "logging.handlers.RotatingFileHandler"
    setup_logging(tmp_path)
    logging.getLogger("t").info("hello-from-test")
    for h in logging.getLogger().handlers:
        h.flush()
    assert "hello-from-test" in (tmp_path / "info.log").read_text()
