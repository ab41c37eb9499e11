"""Debug: train.py under torchrun (1-rank RCCL DDP) with trainer.hip_graph on/off, with/without
validation; prints the epoch logs and the non-finite checkpoint tensors."""
import json, os, socket, subprocess, sys
from pathlib import Path
import torch
ROOT = Path(__file__).resolve().parents[2]
out_dir = Path("/tmp/gdbg")
out_dir.mkdir(parents=True, exist_ok=True)

def port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0)); return s.getsockname()[1]

for graph in (True,):
    for val in (True, False):
        tag = f"g{int(graph)}v{int(val)}"
        cfg = json.loads((ROOT / "config" / "resnet50_bf16.json").read_text())
        cfg["trainer"].update(save_dir=str(out_dir / tag), len_epoch=14, epochs=2, monitor="off", save_period=2,
                              hip_graph=graph, verbosity=2)
        cfg["train_loader"]["args"].update(batch_size=16, num_samples=16 * 14)
        cfg["lr_scheduler"] = {"type": "StepLR", "args": {"step_size": 1, "gamma": 0.5}}
        for k in ("valid_loader", "test_loader"):
            cfg[k]["args"].update(batch_size=16, num_samples=32)
        p = out_dir / f"{tag}.json"
        p.write_text(json.dumps(cfg))
        env = dict(os.environ, PYTHONPATH=str(ROOT), PDT_RUN_ID=tag, HSA_ENABLE_IPC_MODE_LEGACY="0")
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
               "--master-addr=127.0.0.1", f"--master-port={port()}", "train.py", "-c", str(p), "--backend", "native",
               "--seed", "0", "--deterministic"] + ([] if val else ["--no-validate"])
        r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
        o = r.stdout + r.stderr
        print("=====", tag, "rc", r.returncode, flush=True)
        for line in o.splitlines():
            if any(k in line for k in ("loss", "captured", "Error", "Train Epoch")):
                print("   ", line[:200])
        ck = out_dir / tag / cfg["name"] / "train" / tag / "checkpoint-epoch2.pth"
        if ck.exists():
            st = torch.load(ck, weights_only=True, map_location="cpu")["state_dict"]
            bad = [k for k, v in st.items() if v.is_floating_point() and not torch.isfinite(v).all()]
            print("    non-finite:", len(bad), bad[:8], flush=True)
