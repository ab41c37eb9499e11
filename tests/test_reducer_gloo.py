"""The framework's own data-parallel reducer (parallel/reducer.py) on gloo, world 2 (CPU):
gradients equal the single-process full-batch gradients, every gradient lives in its
64-byte-aligned bucket slot, a gradient written into the slot by its producer (what the
native kernels do) is adopted without a copy, an unused parameter reduces as zeros instead of
hanging, and ``no_sync`` accumulates."""
import torch

from test_dist_gloo import _init, _run


class _SlotLinear(torch.autograd.Function):
    """y = x W^T whose weight gradient is written straight into the reducer slot (as the native
    wgrad kernels do through ``grad_out``); records the data pointer it produced."""
    produced = {}

    @staticmethod
    def forward(ctx, x, w):
        ctx.save_for_backward(x, w)
        return x @ w.t()

    @staticmethod
    def backward(ctx, g):
        from pytorch_distributed_template_amd.parallel.reducer import grad_out
        x, w = ctx.saved_tensors
        dw = grad_out(w, *w.shape)
        torch.matmul(g.t(), x, out=dw)
        _SlotLinear.produced[id(w)] = dw.data_ptr()
        return g @ w, dw


class Net(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.conv = torch.nn.Conv2d(3, 4, 3, padding=1)
        self.bn = torch.nn.BatchNorm2d(4)
        self.w = torch.nn.Parameter(torch.randn(5, 4) * 0.3)
        self.fc = torch.nn.Linear(5, 3)
        self.unused = torch.nn.Parameter(torch.ones(7))

    def forward(self, x):
        h = torch.relu(self.bn(self.conv(x))).mean((2, 3))
        return self.fc(_SlotLinear.apply(h, self.w))


def _w_reducer(rank, world, port, q):
    try:
        pdist = _init(rank, world, port)
        from pytorch_distributed_template_amd.parallel.reducer import BucketedDDP, SLOT_ALIGN
        torch.manual_seed(0)
        model, ref = Net(), Net()
        ref.load_state_dict(model.state_dict())
        dp = BucketedDDP(model, torch.device("cpu"), bucket_cap_mb=0.0001, first_bucket_mb=0.00001)
        torch.manual_seed(1)
        X = torch.randn(8, 3, 6, 6)
        Y = torch.randint(0, 3, (8,))
        xs, ys = X[rank * 4:(rank + 1) * 4], Y[rank * 4:(rank + 1) * 4]
        out = {}
        torch.nn.functional.cross_entropy(dp(xs), ys).backward()
        # reference: the full batch in one process, BN statistics per shard (as DDP without SyncBN)
        loss = sum(torch.nn.functional.cross_entropy(ref(X[r * 4:(r + 1) * 4]), Y[r * 4:(r + 1) * 4])
                   for r in range(world)) / world
        loss.backward()
        pr = dict(ref.named_parameters())
        out["diff"] = max(float((p.grad - pr[n].grad).abs().max()) for n, p in model.named_parameters()
                          if n != "unused")
        out["unused_zero"] = bool((model.unused.grad == 0).all())
        flats = {b.flat.data_ptr(): b.flat for b in dp.buckets}
        ok = True
        for p in model.parameters():
            b = dp.buckets[dp._bucket_of[id(p)]].flat
            off = (p.grad.data_ptr() - b.data_ptr()) // 4
            ok &= 0 <= off < b.numel() and off % SLOT_ALIGN == 0
        out["in_slots"] = bool(ok) and len(flats) == len(dp.buckets) and len(dp.buckets) > 2
        out["adopted"] = model.w.grad.data_ptr() == _SlotLinear.produced[id(model.w)]
        # no_sync: two local backwards, then a synced one -> 3 x the averaged gradient of one batch
        g1 = model.fc.weight.grad.clone()
        for p in model.parameters():
            p.grad = None
        with dp.no_sync():
            torch.nn.functional.cross_entropy(dp(xs), ys).backward()
            torch.nn.functional.cross_entropy(dp(xs), ys).backward()
        torch.nn.functional.cross_entropy(dp(xs), ys).backward()
        out["nosync"] = float((model.fc.weight.grad - 3 * g1).abs().max())
        q.put((rank, out))
        pdist.cleanup()
    except Exception as e:  # pragma: no cover
        import traceback
        q.put((rank, repr(e) + traceback.format_exc()))


def _w_accumulate(rank, world, port, q):
    """Retained gradients: ``zero_grad(set_to_none=False)`` and ``no_sync`` micro-batches on
    DIFFERENT batches must sum exactly as a single process does -- checked on the slot-written
    ``w`` (the native-kernel path) as well as on the stock-op parameters."""
    try:
        pdist = _init(rank, world, port)
        from pytorch_distributed_template_amd.parallel.reducer import BucketedDDP
        torch.manual_seed(0)
        model, ref = Net(), Net()
        ref.load_state_dict(model.state_dict())
        for m in (model, ref):
            m.bn.eval()  # batch-independent normalisation: sums over micro-batches are exact
        dp = BucketedDDP(model, torch.device("cpu"), bucket_cap_mb=0.0001, first_bucket_mb=0.00001)
        torch.manual_seed(1)
        batches = [(torch.randn(8, 3, 6, 6), torch.randint(0, 3, (8,))) for _ in range(3)]
        shard = lambda b: (b[0][rank * 4:(rank + 1) * 4], b[1][rank * 4:(rank + 1) * 4])  # noqa: E731
        ce = torch.nn.functional.cross_entropy

        def ref_grads(bs):
            for p in ref.parameters():
                p.grad = None
            for X, Y in bs:
                (sum(ce(ref(X[r * 4:(r + 1) * 4]), Y[r * 4:(r + 1) * 4]) for r in range(world)) / world).backward()
            return {n: p.grad.clone() for n, p in ref.named_parameters() if n != "unused"}

        def diff(want):
            return max(float((p.grad - want[n]).abs().max()) for n, p in model.named_parameters() if n != "unused")

        out = {}
        # (a) retained gradients zeroed in place between steps (the HIP-graph trainer's old path)
        opt = torch.optim.SGD(model.parameters(), lr=0.0)
        ce(dp(shard(batches[0])[0]), shard(batches[0])[1]).backward()
        opt.zero_grad(set_to_none=False)
        ce(dp(shard(batches[1])[0]), shard(batches[1])[1]).backward()
        out["zero_inplace"] = diff(ref_grads([batches[1]]))
        out["w_ratio"] = float(model.w.grad.norm() / ref.w.grad.norm())
        # (b) no_sync accumulation over three different batches
        for p in model.parameters():
            p.grad = None
        with dp.no_sync():
            ce(dp(shard(batches[0])[0]), shard(batches[0])[1]).backward()
            ce(dp(shard(batches[1])[0]), shard(batches[1])[1]).backward()
        ce(dp(shard(batches[2])[0]), shard(batches[2])[1]).backward()
        out["nosync"] = diff(ref_grads(batches))
        # (c) a backward that raised before its final callback does not wedge the next step,
        # and an all-reduce it left in flight on a bucket finishes before the next backward
        # writes that bucket's slots (forward waits for it)
        dp._in_backward = True
        for b in dp.buckets:
            b.flat.fill_(1e6)
            b.work = torch.distributed.all_reduce(b.flat, async_op=True)
        for p in model.parameters():
            p.grad = None
        ce(dp(shard(batches[2])[0]), shard(batches[2])[1]).backward()
        out["after_abort"] = diff(ref_grads([batches[2]]))
        out["works_cleared"] = all(b.work is None for b in dp.buckets)
        q.put((rank, out))
        pdist.cleanup()
    except Exception as e:  # pragma: no cover
        import traceback
        q.put((rank, repr(e) + traceback.format_exc()))


def test_reducer_accumulates_into_retained_gradients():
    res = _run(_w_accumulate)
    for r in (0, 1):
        o = res[r]
        assert isinstance(o, dict), o
        assert o["zero_inplace"] < 1e-6 and abs(o["w_ratio"] - 1) < 1e-6, o
        assert o["nosync"] < 1e-6, o
        assert o["after_abort"] < 1e-6 and o["works_cleared"], o


class _ManyParams(torch.nn.Module):
    """More than 4 096 parameters; on rank 1 the LAST one has another shape (same numel)."""

    def __init__(self, odd):
        super().__init__()
        self.ps = torch.nn.ParameterList([torch.nn.Parameter(torch.zeros(2)) for _ in range(5000)])
        self.ps.append(torch.nn.Parameter(torch.zeros(1, 2) if odd else torch.zeros(2)))


def _w_shape_mismatch(rank, world, port, q):
    try:
        pdist = _init(rank, world, port)
        from pytorch_distributed_template_amd.parallel.reducer import BucketedDDP
        try:
            BucketedDDP(_ManyParams(odd=rank == 1), torch.device("cpu"))
            q.put((rank, {"msg": "constructed"}))
        except RuntimeError as e:
            q.put((rank, {"msg": "raised: " + str(e)}))
        pdist.cleanup()
    except Exception as e:  # pragma: no cover
        import traceback
        q.put((rank, repr(e) + traceback.format_exc()))


def test_reducer_shape_check_covers_every_parameter_and_raises_on_every_rank():
    """The signature covers all parameters (a mismatch at index 5 000 is found) and a mismatch
    raises on EVERY rank, rank 0 included (else rank 0 would wait in the parameter broadcast)."""
    res = _run(_w_shape_mismatch)
    for r in (0, 1):
        assert res[r]["msg"].startswith("raised: BucketedDDP: parameter shapes differ"), res[r]


def test_reducer_matches_single_process_and_uses_slots():
    res = _run(_w_reducer)
    for r in (0, 1):
        o = res[r]
        assert o["diff"] < 1e-5, o
        assert o["unused_zero"] and o["in_slots"] and o["adopted"], o
        assert o["nosync"] < 1e-5, o


def test_plan_buckets_small_last_bucket():
    """The last bucket is split so that only the gradients produced last (<= last_bucket_mb: the
    stem and first stage of ResNet-50) stay exposed after backward."""
    from pytorch_distributed_template_amd import models
    from pytorch_distributed_template_amd.parallel.reducer import plan_buckets
    ps = [p for p in models.resnet50(num_classes=1000).parameters() if p.requires_grad]
    mib = lambda b: sum(ps[i].numel() * 4 for i in b) / 2 ** 20  # noqa: E731
    plain = plan_buckets(ps, 64.0, 8.0)
    split = plan_buckets(ps, 64.0, 8.0, 4.0)
    assert len(split) == len(plain) + 1
    assert mib(split[-1]) <= 4.0 and 0 in split[-1]  # the stem conv (registered first) is in the tail
    assert sorted(i for b in split for i in b) == list(range(len(ps)))
    assert split[:-2] == plain[:-1] and split[-2] + split[-1] == plain[-1]
