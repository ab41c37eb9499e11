"""Quick probe: stock PyTorch-ROCm ResNet-50 bf16 training throughput on one GPU."""
import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn.functional as F
from pytorch_distributed_template_amd.models.resnet import resnet50
from pytorch_distributed_template_amd.ops import fused
fused.set_backend("torch")

bs = int(os.environ.get("BS", 256))
steps = int(os.environ.get("STEPS", 20))
mode = os.environ.get("MODE", "autocast")
torch.backends.cudnn.benchmark = True
dev = torch.device("cuda")
model = resnet50().to(dev).to(memory_format=torch.channels_last)
if mode == "bf16":
    model = model.to(torch.bfloat16)
opt = torch.optim.SGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=5e-5)
x = torch.randn(bs, 3, 224, 224, device=dev).to(memory_format=torch.channels_last)
if mode == "bf16":
    x = x.to(torch.bfloat16)
y = torch.randint(0, 1000, (bs,), device=dev)

def step():
    opt.zero_grad(set_to_none=True)
    with torch.autocast("cuda", dtype=torch.bfloat16, enabled=(mode == "autocast")):
        out = model(x)
        loss = F.cross_entropy(out, y)
    loss.backward()
    opt.step()
    return loss

for _ in range(5):
    step()
torch.cuda.synchronize()
t = time.time()
for _ in range(steps):
    step()
torch.cuda.synchronize()
dt = (time.time() - t) / steps
print(f"mode={mode} bs={bs} ms/step={dt*1e3:.2f} img/s={bs/dt:.1f} maxmem={torch.cuda.max_memory_allocated()/2**30:.1f}GiB", flush=True)
