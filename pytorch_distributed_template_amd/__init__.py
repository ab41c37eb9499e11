"""MI355X-native config-driven distributed training template.

Same CLI / config schema / checkpoint format as Yun-960/Pytorch-Distributed-Template
(``train.py``, ``test.py``, ``config/*.json``); hand-written HIP/CDNA4 kernels
(``csrc/``) for the image-classification hot path; DDP over RCCL/xGMI.
"""
__version__ = "0.1.0"
