"""DDP over a real RCCL process group on the test box's one MI355X.

The reference's only parallel machinery is ``init_process_group('nccl')`` + DDP
(/root/reference/train.py:25-28,45-52). These tests run exactly that path at
world size 1 -- RCCL communicator, DDP reducer, bucket views, RCCL all-reduce
on the reducer's stream, comm hooks -- under ``torchrun --nproc-per-node 1``
and in a spawned 1-rank job, with the native HIP kernels doing every op:

* the DDP-wrapped gradients equal the unwrapped ones (fp32 buckets: bitwise;
  the bf16 comm hook: the bf16 rounding of them), and FusedSGD stepping on the
  bucket views gives the same weights as on plain gradients;
* ``train.py`` -> resume -> ``test.py`` of the ResNet-50 bf16 config under
  torchrun (backend reported as ``nccl``).
"""
import json
import os
import socket
import subprocess
import sys
from pathlib import Path

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(port, hook, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1",
                          LOCAL_RANK="0")
        import torch.distributed as dist
        from pytorch_distributed_template_amd.models import resnet50
        from pytorch_distributed_template_amd.ops import fused
        from pytorch_distributed_template_amd.optim import FusedSGD
        from pytorch_distributed_template_amd.parallel import wrap_ddp
        from pytorch_distributed_template_amd.utils import dist as pdist
        dev = pdist.init_distributed()
        assert dist.is_initialized() and dist.get_backend() == "nccl" and dist.get_world_size() == 1
        fused.set_backend("native")
        torch.manual_seed(0)
        model = resnet50(num_classes=16).to(dev).to(memory_format=torch.channels_last)
        ref = resnet50(num_classes=16).to(dev).to(memory_format=torch.channels_last)
        ref.load_state_dict(model.state_dict())
        g = torch.Generator(device="cpu").manual_seed(7)
        x = torch.randn(8, 3, 64, 64, generator=g).to(dev).to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        y = torch.randint(0, 16, (8,), generator=g).to(dev)
        fused.softmax_cross_entropy(ref(x), y).backward()
        ddp = wrap_ddp(model, dev, bucket_cap_mb=8, broadcast_buffers=True, gradient_as_bucket_view=True,
                       comm_hook=hook)
        assert type(ddp).__name__ == ("DistributedDataParallel" if hook else "BucketedDDP")
        fused.softmax_cross_entropy(ddp(x), y).backward()
        torch.cuda.synchronize()
        errs, views = [], 0
        for p, r in zip(model.parameters(), ref.parameters()):
            want = r.grad if hook is None else r.grad.to(torch.bfloat16).float()
            errs.append(float((p.grad - want).abs().max() / want.abs().max().clamp_min(1e-12)))
            # gradients live in the buckets: torch DDP (gradient_as_bucket_view) hands out bucket
            # views; the native reducer's slots are adopted by autograd through detach(), which
            # shares the storage without keeping ``_base`` -- check the address instead
            if hook is None:
                views += int(any(b.flat.data_ptr() <= p.grad.data_ptr() <
                                 b.flat.data_ptr() + b.flat.numel() * b.flat.element_size() for b in ddp.buckets))
            else:
                views += int(p.grad._base is not None)
        # FusedSGD on the bucket views == FusedSGD on plain gradients (same grads in)
        if hook is None:
            o1 = FusedSGD(list(model.parameters()), lr=0.1, momentum=0.9, weight_decay=1e-4)
            o2 = FusedSGD(list(ref.parameters()), lr=0.1, momentum=0.9, weight_decay=1e-4)
            o1.step()
            o2.step()
            torch.cuda.synchronize()
            werr = max(float((a - b).abs().max()) for a, b in zip(model.parameters(), ref.parameters()))
        else:
            werr = 0.0
        # the native reducer: every gradient was written into its bucket slot by the kernel that
        # produced it (no per-parameter copy / scale launches)
        copies = getattr(ddp, "fallback_copies", 0)
        # a plain RCCL all-reduce on the same communicator
        t = torch.full((1024,), 3.0, device=dev)
        dist.all_reduce(t)
        torch.cuda.synchronize()
        q.put((max(errs), views, werr, float(t.sum()), copies))
        dist.destroy_process_group()
    except Exception:  # pragma: no cover
        import traceback
        q.put(traceback.format_exc())


@pytest.mark.parametrize("hook", [None, "bf16"])
def test_rccl_one_rank_ddp_native_grads(hook):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(_port(), hook, q))
    p.start()
    res = q.get(timeout=300)
    p.join(60)
    assert not isinstance(res, str), res
    err, views, werr, tsum, copies = res
    assert views > 100, views
    assert copies == 0, copies
    assert tsum == 3.0 * 1024
    if hook is None:
        assert err == 0.0, err      # 1 rank, fp32 buckets: the all-reduce is exact
        assert werr == 0.0, werr    # FusedSGD on bucket views
    else:
        assert err < 1e-2, err      # bf16-compressed buckets


def _vit_worker(port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1",
                          LOCAL_RANK="0")
        from pytorch_distributed_template_amd.models.vit import VisionTransformer
        from pytorch_distributed_template_amd.ops import fused
        from pytorch_distributed_template_amd.parallel import wrap_ddp
        from pytorch_distributed_template_amd.utils import dist as pdist
        dev = pdist.init_distributed()
        fused.set_backend("native")
        torch.manual_seed(0)
        model = VisionTransformer(depth=2, fp8=True).to(dev).to(memory_format=torch.channels_last)
        ddp = wrap_ddp(model, dev, bucket_cap_mb=8, broadcast_buffers=True, gradient_as_bucket_view=True)
        x = torch.randn(8, 3, 224, 224, device=dev)
        y = torch.randint(0, 1000, (8,), device=dev)
        for _ in range(3):  # the fp8 scaling state (and the fused bias-gradient paths) settle
            model.zero_grad(set_to_none=True)
            fused.softmax_cross_entropy(ddp(x), y).backward()
        torch.cuda.synchronize()
        q.put((ddp.fallback_copies, sorted(ddp.fallback_shapes)))
        import torch.distributed as dist
        dist.destroy_process_group()
    except Exception:  # pragma: no cover
        import traceback
        q.put(traceback.format_exc())


def test_rccl_one_rank_ddp_vit_fp8_grads_in_slots():
    """The fp8 ViT under the native reducer: every gradient but the two the stock ops of the
    patch-embedding assembly produce (class token, position embedding) is written into its
    bucket slot -- including the bias gradients of the attention projection and fc2, which
    the LayerNorm backward forms and hands over (``_pdt_db``)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_vit_worker, args=(_port(), q))
    p.start()
    res = q.get(timeout=300)
    p.join(60)
    assert not isinstance(res, str), res
    copies, shapes = res
    assert set(shapes) <= {(1, 1, 768), (1, 197, 768)}, shapes
    assert copies <= 2 * 3, copies


def test_resnet50_config_torchrun_rccl_train_resume_test(tmp_path):
    cfg = json.loads((ROOT / "config" / "resnet50_bf16.json").read_text())
    cfg["trainer"].update(save_dir=str(tmp_path), len_epoch=2, epochs=1, monitor="max val_accuracy")
    cfg["train_loader"]["args"].update(batch_size=32, num_samples=64)
    for k in ("valid_loader", "test_loader"):
        cfg[k]["args"].update(batch_size=32, num_samples=48)
    p = tmp_path / "cfg.json"
    p.write_text(json.dumps(cfg))
    env = dict(os.environ, PYTHONPATH=str(ROOT), PDT_RUN_ID="t1", HSA_ENABLE_IPC_MODE_LEGACY="0")

    def run(args):
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
               "--master-addr=127.0.0.1", f"--master-port={_port()}"] + args
        r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
        assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
        return r.stdout + r.stderr

    out = run(["train.py", "-c", str(p), "--backend", "native"])
    assert "process group: nccl, world size 1" in out, out[-3000:]
    assert "BucketedDDP(" in out  # the model print is the data-parallel wrapper
    ck = tmp_path / cfg["name"] / "train" / "t1" / "checkpoint-epoch1.pth"
    assert ck.exists(), out[-3000:]
    state = torch.load(ck, weights_only=True, map_location="cpu")
    assert state["arch"] == "ResNet50" and not any(k.startswith("module.") for k in state["state_dict"])
    env["PDT_RUN_ID"] = "t2"
    out = run(["train.py", "-r", str(ck), "--epochs", "2", "--backend", "native"])
    assert "Resume training from epoch 2" in out
    ck2 = tmp_path / cfg["name"] / "train" / "t2" / "checkpoint-epoch2.pth"
    assert ck2.exists(), out[-3000:]
    env["PDT_RUN_ID"] = "t3"
    out = run(["test.py", "-r", str(ck2), "--backend", "native"])
    assert "'loss':" in out and "'accuracy':" in out
