"""MI355X end-to-end (SURVEY §7.3 slice B): ResNet-50 bf16 config through
train.py (native kernels, device-resident synthetic loader, DDP world 1 over
RCCL) -> checkpoint -> test.py; and the synthetic loader's native fill."""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]


def test_synthetic_loader_native_fill():
    from pytorch_distributed_template_amd.data import SyntheticImageNetLoader
    dl = SyntheticImageNetLoader(batch_size=8, num_samples=20, pool=2, training=False)
    xs = [x for x, _ in dl]
    assert [x.shape[0] for x in xs] == [8, 8, 4]
    x = xs[0]
    assert x.is_cuda and x.dtype == torch.bfloat16
    # 3-channel images live in NHWC storage zero-padded to 4 channels (the space-to-depth
    # stem GEMM reads 16-B pairs of pixels in place); the [B, 3, H, W] tensor is a view into it
    from pytorch_distributed_template_amd.ops import native_ops
    xp = native_ops.nhwc_padded_view(x, 4)
    assert xp is not None and xp.is_contiguous(memory_format=torch.channels_last)
    assert torch.equal(xp[:, :3], x) and not xp[:, 3:].any()
    assert -1.0 <= float(x.min()) and float(x.max()) <= 1.0 and float(x.float().std()) > 0.5
    dl2 = SyntheticImageNetLoader(batch_size=8, num_samples=20, pool=2, training=False)
    assert torch.equal(next(iter(dl2))[0], x)  # counter-based: same seed -> same data


def test_synthetic_imagenet_kernel_matches_host_hash():
    """pdt_synth_images_bf16 == the torch-integer-op host path, bit for bit (images and labels)."""
    from pytorch_distributed_template_amd.data.synthetic import SyntheticImageNet
    g = SyntheticImageNet(1000, image_size=16, num_classes=11, seed=9, device="cuda")
    c = SyntheticImageNet(1000, image_size=16, num_classes=11, seed=9, device="cpu", dtype="bfloat16")
    idx = [3, 999, 0, 512, 77]
    xg, yg = g.collate(idx)
    xc, yc = c.collate(idx)
    assert getattr(xg, "pdt_nhwc_pad", None) == 4
    assert torch.equal(xg.cpu(), xc) and torch.equal(yg.cpu(), yc)


def test_resnet50_config_train_resume_test(tmp_path):
    cfg = json.loads((ROOT / "config" / "resnet50_bf16.json").read_text())
    cfg["trainer"].update(save_dir=str(tmp_path), len_epoch=3, epochs=1, monitor="max val_accuracy")
    cfg["train_loader"]["args"].update(batch_size=32, num_samples=96)
    for k in ("valid_loader", "test_loader"):
        cfg[k]["args"].update(batch_size=32, num_samples=48)
    p = tmp_path / "cfg.json"
    p.write_text(json.dumps(cfg))
    env = dict(os.environ, PYTHONPATH=str(ROOT), PDT_RUN_ID="g1")

    def run(args):
        r = subprocess.run([sys.executable] + args, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
        assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
        return r.stdout + r.stderr

    out = run(["train.py", "-c", str(p), "--backend", "native"])
    run_dir = tmp_path / cfg["name"] / "train" / "g1"
    ck = run_dir / "checkpoint-epoch1.pth"
    assert ck.exists(), out
    state = torch.load(ck, weights_only=True, map_location="cpu")
    assert state["arch"] == "ResNet50" and torch.isfinite(state["state_dict"]["fc.weight"]).all()
    assert "val_loss" in out
    env["PDT_RUN_ID"] = "g2"
    out = run(["test.py", "-r", str(ck), "--backend", "native"])
    assert "'loss':" in out and "'accuracy':" in out
