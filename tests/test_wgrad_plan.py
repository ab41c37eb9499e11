"""Split planning of the fp8 weight gradient (csrc/wgrad_f8.hip pdt_wgrad_f8_plan): the split
count minimises (dispatch waves) x (k-tiles per split) for the device's resident workgroups, so
a grid never ends one straggler workgroup past a full wave (the old ceil(target / tiles) gave
the ViT qkv shape 513 workgroups = 3 waves on 256 CUs). Host-side arithmetic only: on a machine
without a GPU the occupancy query falls back to 1 workgroup per CU on 256 CUs -- the MI355X
value for these one-workgroup-per-CU tiles."""
import ctypes

import pytest

from pytorch_distributed_template_amd.ops import native_ops as no

if not no._LIB_PATH.exists():
    pytest.skip("native kernel library not built (python -m pytorch_distributed_template_amd.ops.build)",
                allow_module_level=True)

M = 1024 * 197  # ViT-B/16 batch 1024 tokens
BK = 128        # token rows per k-tile


def plan(Mo, No, v):
    kps = ctypes.c_int(0)
    s = no._load().pdt_wgrad_f8_plan(M, Mo, No, v, ctypes.byref(kps))
    return s, kps.value


def test_plan_fills_whole_waves_for_the_vit_shapes():
    nk = -(-M // BK)
    for Mo, No, v in [(2304, 768, 12), (768, 768, 10), (3072, 768, 12), (768, 3072, 10)]:
        s, kps = plan(Mo, No, v)
        tiles = -(-Mo // 256) * -(-No // 256)
        assert s * kps >= nk > (s - 1) * kps, (Mo, No)      # the splits cover every k-tile once
        wgs = tiles * s
        waves = -(-wgs // 256)
        assert wgs > (waves - 1) * 256 + 256 // 2, (Mo, No, wgs)  # the last wave is mostly full
        assert kps * BK >= 512                                # >= 512 token rows per split


def test_plan_qkv_shape_is_one_wave():
    s, kps = plan(2304, 768, 12)  # 27 tiles: 9 splits x 176 k-tiles = 243 workgroups, one wave
    assert (s, kps) == (9, 176)
