"""Metric registry (``"metrics"`` list in config). Reference: ``/root/reference/model/metric.py:4-20``.

Same semantics (fraction of correct argmax / top-k over a batch) and same
Python-float return. The ``*_count`` variants return device tensors of
correct-counts so callers can accumulate without a host sync per batch.
"""
import torch


def correct_count(output, target):
    with torch.no_grad():
        return (torch.argmax(output, dim=1) == target).sum()


def topk_correct_count(output, target, k=3):
    with torch.no_grad():
        pred = torch.topk(output, k, dim=1)[1]
        return (pred == target.unsqueeze(1)).any(dim=1).sum()


def accuracy(output, target):
    assert output.shape[0] == len(target)
    return correct_count(output, target).item() / len(target)


def top_k_acc(output, target, k=3):
    assert output.shape[0] == len(target)
    return topk_correct_count(output, target, k).item() / len(target)
