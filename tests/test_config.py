"""ConfigParser: CLI overrides, run-dir layout, factory, resume/fine-tune merge
(reference: /root/reference/parse_config.py)."""
import argparse
import collections
import json

import pytest
import torch

from pytorch_distributed_template_amd.config import ConfigParser, _get_opt_name
from pytorch_distributed_template_amd.utils import read_json, write_json

CustomArgs = collections.namedtuple("CustomArgs", "flags type target")


def _cfg(tmp_path):
    return {
        "name": "T",
        "arch": {"type": "MnistModel", "args": {}},
        "train_loader": {"type": "X", "args": {"batch_size": 4}},
        "optimizer": {"type": "SGD", "args": {"lr": 0.1}},
        "loss": "nll_loss",
        "metrics": ["accuracy"],
        "trainer": {"epochs": 1, "save_dir": str(tmp_path / "ck"), "save_period": 1, "verbosity": 2,
                    "monitor": "off", "tensorboard": False},
    }


def _parser():
    p = argparse.ArgumentParser()
    p.add_argument("-c", "--config", default=None)
    p.add_argument("-r", "--resume", default=None)
    p.add_argument("-s", "--save_dir", default=None)
    return p


def test_from_args_overrides_and_run_dir(tmp_path, monkeypatch):
    cfgp = tmp_path / "c.json"
    write_json(_cfg(tmp_path), cfgp)
    opts = [CustomArgs(["--lr", "--learning_rate"], float, "optimizer;args;lr"),
            CustomArgs(["--bs", "--batch_size"], int, "train_loader;args;batch_size")]
    monkeypatch.setattr("sys.argv", ["x", "-c", str(cfgp), "--lr", "0.5", "--bs", "32"])
    args, cfg = ConfigParser.from_args(_parser(), opts, run_id="RUN1")
    assert cfg["optimizer"]["args"]["lr"] == 0.5
    assert cfg["train_loader"]["args"]["batch_size"] == 32  # reference's --bs hit a KeyError (Q3)
    assert cfg.save_dir == tmp_path / "ck" / "T" / "train" / "RUN1"
    saved = read_json(cfg.save_dir / "config.json")
    assert saved["optimizer"]["args"]["lr"] == 0.5
    assert cfg.log_dir == cfg.save_dir


def test_test_mode_dir_and_save_dir_override(tmp_path, monkeypatch):
    cfgp = tmp_path / "c.json"
    write_json(_cfg(tmp_path), cfgp)
    monkeypatch.setattr("sys.argv", ["x", "-c", str(cfgp), "-s", str(tmp_path / "other")])
    _, cfg = ConfigParser.from_args(_parser(), [], training=False, run_id="R")
    assert cfg.save_dir == tmp_path / "other" / "T" / "test" / "R"


def test_resume_loads_ckpt_config_and_finetune_merge(tmp_path, monkeypatch):
    run = tmp_path / "run"
    run.mkdir()
    base = _cfg(tmp_path)
    write_json(base, run / "config.json")
    (run / "checkpoint-epoch1.pth").write_bytes(b"")
    ft = {"optimizer": {"type": "Adam", "args": {"lr": 1e-4}}}
    write_json(ft, tmp_path / "ft.json")
    monkeypatch.setattr("sys.argv", ["x", "-r", str(run / "checkpoint-epoch1.pth"), "-c", str(tmp_path / "ft.json")])
    _, cfg = ConfigParser.from_args(_parser(), [], run_id="R2")
    assert cfg.resume == run / "checkpoint-epoch1.pth"
    assert cfg["optimizer"]["type"] == "Adam"        # shallow top-level update
    assert cfg["arch"]["type"] == "MnistModel"


def test_init_obj_and_ftn(tmp_path):
    cfg = ConfigParser(_cfg(tmp_path), run_id="R3")
    lin = torch.nn.Linear(2, 2)
    opt = cfg.init_obj("optimizer", torch.optim, lin.parameters())
    assert isinstance(opt, torch.optim.SGD) and opt.param_groups[0]["lr"] == 0.1
    with pytest.raises(AssertionError):
        cfg.init_obj("optimizer", torch.optim, lin.parameters(), lr=0.2)
    from pytorch_distributed_template_amd import optim as pdt_optim
    cfg.config["optimizer"]["type"] = "FusedSGD"
    o2 = cfg.init_obj("optimizer", [pdt_optim, torch.optim], lin.parameters())
    assert type(o2).__name__ == "FusedSGD"
    f = cfg.init_ftn("optimizer", [pdt_optim, torch.optim])
    assert type(f(lin.parameters())).__name__ == "FusedSGD"
    d = cfg.to_dict()
    assert isinstance(d, dict) and json.dumps(d)


def test_opt_name():
    assert _get_opt_name(["--lr", "--learning_rate"]) == "lr"
    assert _get_opt_name(["-x", "--batch-size"]) == "batch_size"


def test_get_logger_verbosity(tmp_path):
    cfg = ConfigParser(_cfg(tmp_path), run_id="R4")
    assert cfg.get_logger("a", 0).level == 30
    with pytest.raises(AssertionError):
        cfg.get_logger("a", 7)
