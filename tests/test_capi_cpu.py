"""The C-ABI library loads on a GPU-less host and exports every entry point
include/ngp_amd.h declares; argument checks fail loudly like the
reference's CHECK_INPUT (no compute is launched here)."""
import ctypes
import os
import re

import pytest
import torch

import hashgrid as HG
import oracle as O
import vren

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    hdr = open(os.path.join(ROOT, "include", "ngp_amd.h")).read()
    hdr = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
    return sorted(set(re.findall(r"\b(ngp_[a-z0-9_]+)\s*\(", hdr)))


def test_header_declares_the_vren_surface():
    names = _declared()
    for n in ("ngp_ray_aabb_intersect", "ngp_morton3d", "ngp_morton3d_invert", "ngp_packbits",
              "ngp_march_train_count", "ngp_march_train_write", "ngp_march_test", "ngp_composite_train_fw",
              "ngp_composite_train_bw", "ngp_composite_test_fw", "ngp_field_forward", "ngp_field_backward"):
        assert n in names


def test_library_exports_every_declared_symbol():
    L = vren.lib()
    missing = [n for n in _declared() if not hasattr(L, n)]
    assert not missing, missing
    assert L.ngp_version().startswith(b"ngp_amd")


def test_every_declared_function_has_a_ctypes_signature():
    """An undeclared argtypes list lets ctypes pass Python ints as 32-bit C ints
    and floats not at all: every C-ABI entry point must be declared."""
    import hashgrid as HG
    L = HG._lib()
    missing = [n for n in _declared() if n != "ngp_version" and getattr(L, n).argtypes is None]
    assert not missing, missing


def test_library_levels_equal_oracle_levels():
    for scale in (0.5, 16.0):
        g = HG.HashGrid(scale)
        spec = O.HashGridSpec(16, 19, 16, scale=scale)
        assert g.resolutions == spec.res.tolist() and g.offsets == spec.offsets.tolist()
        assert list(g.desc.scales)[:16] == spec.scales.tolist()


def test_cpu_tensors_are_rejected_like_check_input():
    x = torch.zeros(4, 3)
    with pytest.raises(RuntimeError, match="rays_o must be a CUDA tensor"):
        vren.ray_aabb_intersect(x, x, torch.zeros(1, 3), torch.ones(1, 3), 1)
    with pytest.raises(RuntimeError, match="coords must be a CUDA tensor"):
        vren.morton3D(x.int())


def test_bad_arguments_return_einval():
    L = vren.lib()
    # null pointers with a non-zero size: rejected before any launch
    assert L.ngp_morton3d(None, 10, None, None) == -1
    assert L.ngp_composite_train_fw(None, None, None, None, None, 5, 1e-4, None, None, None, None, None, None) == -1
    assert L.ngp_march_test(None, None, None, None, 1, None, 1, 128, 0.5, 0.0, 1, 1024, None, None, None, None, None,
                            None, None) == -1
    assert L.ngp_bitfield_summary(None, 256, 128, None, None) == -1
    # zero-size calls are no-ops
    assert L.ngp_morton3d(None, 0, None, None) == 0


def test_new_entry_points_reject_bad_arguments_without_launching():
    """Argument checks run before any launch (no GPU needed): NGP_EINVAL (-1)."""
    import ctypes as C
    L = HG._lib()
    assert L.ngp_render_test_capacity(-1, 1) == -1 and L.ngp_render_test_capacity(10, 4) == 40
    assert L.ngp_render_test_begin(-1, None, None, None, None, None, None) == -1
    assert L.ngp_render_test_begin(4, None, None, None, None, None, None) == -1
    assert L.ngp_render_test_composite(None, None, None, None, None, 4, 2, None, None, None, C.c_float(1e-4),
                                       None, None, None, None) == -1
    assert L.ngp_render_test_finish(None, 4, None, None, None) == -1
    assert L.ngp_distortion_loss_fw(None, None, None, None, -1, None, None, None, None) == -1
    assert L.ngp_distortion_loss_fw(None, None, None, None, 3, None, None, None, None) == -1
    assert L.ngp_distortion_loss_bw(None, None, None, None, None, None, None, 3, None, None) == -1
    assert L.ngp_distortion_loss_fw(None, None, None, None, 0, None, None, None, None) == 0  # empty: no-op
    g = HG.HashGrid(0.5)
    assert L.ngp_density_input_grad(None, 5, C.byref(g.desc), None, None, None, None, None) == -1


def test_gradient_replica_entry_points_check_arguments_without_launching():
    """ngp_hash_backward_levels_rep / ngp_hash_backward_rep_floats /
    ngp_adam_step_dev_rep: sizes and
    argument checks on the host, before any launch (NGP_EINVAL = -1)."""
    import ctypes as C
    L = HG._lib()
    g = HG.HashGrid(0.5)
    d = C.byref(g.desc)
    assert L.ngp_hash_backward_rep_floats(d, 4, 8) == 8 * 2 * g.offsets[4]
    assert L.ngp_hash_backward_rep_floats(d, 0, 8) == 0
    assert L.ngp_hash_backward_rep_floats(d, 17, 8) == 0 and L.ngp_hash_backward_rep_floats(d, 4, 0) == 0
    p = C.c_void_p(16)  # never dereferenced: every call below fails its checks first
    # replicas beyond the atomic levels, replica count 0 / > 64, negative n
    assert L.ngp_hash_backward_levels_rep(p, 10, None, None, d, p, p, 0, 8, p, 9, 8, 1, None) == -1
    assert L.ngp_hash_backward_levels_rep(p, 10, None, None, d, p, p, 0, 8, p, 4, 0, 1, None) == -1
    assert L.ngp_hash_backward_levels_rep(p, 10, None, None, d, p, p, 0, 8, p, 4, 65, 1, None) == -1
    assert L.ngp_hash_backward_levels_rep(p, -1, None, None, d, p, p, 0, 8, p, 4, 8, 1, None) == -1
    f = C.c_float
    # replica range not a multiple of 4, past the Adam range, misaligned replicas
    assert L.ngp_adam_step_dev_rep(p, p, p, p, p, 64, p, f(0.9), f(0.999), f(1e-15), p, f(1.0), 1, p, 2, 8, 8,
                                   None) == -1
    assert L.ngp_adam_step_dev_rep(p, p, p, p, p, 64, p, f(0.9), f(0.999), f(1e-15), p, f(1.0), 1, p, 0, 68, 8,
                                   None) == -1
    assert L.ngp_adam_step_dev_rep(p, p, p, p, p, 64, p, f(0.9), f(0.999), f(1e-15), p, f(1.0), 1, C.c_void_p(20),
                                   0, 8, 8, None) == -1



def test_row_forward_entry_points_check_arguments_without_launching():
    """ngp_field_forward_first / ngp_rays_nonempty
    (round 4): argument checks on the host, before any launch (NGP_EINVAL =
    -1); zero rows are a no-op."""
    import ctypes as C
    L, Lv = HG._lib(), vren.lib()
    g = HG.HashGrid(0.5)
    d = C.byref(g.desc)
    p = C.c_void_p(256)  # never dereferenced: every call below fails its checks first (or has nothing to do)
    f = C.c_float(1e-4)
    # neither the counts nor the round-2 list asked for; the list without its length; a misaligned length
    assert L.ngp_field_forward_first(p, p, p, p, None, None, 8, 64, f, d, p, p, p, p, p, None, None, None, None,
                                     None) == -1
    assert L.ngp_field_forward_first(p, p, p, p, None, None, 8, 64, f, d, p, p, p, p, p, None, p, None, None,
                                     None) == -1
    assert L.ngp_field_forward_first(p, p, p, p, None, None, 8, 64, f, d, p, p, p, p, p, None, p, C.c_void_p(260),
                                     None, None) == -1
    assert L.ngp_field_forward_first(None, None, None, None, None, None, -1, 64, f, d, None, None, None, None, None,
                                     None, None, None, None, None) == -1
    assert L.ngp_field_forward_first(None, None, None, None, None, None, 0, 64, f, d, None, None, None, None, None,
                                     None, None, None, None, None) == 0
    assert Lv.ngp_rays_nonempty(p, 8, None, p, None, None, None) == -1
    assert Lv.ngp_rays_nonempty(p, -1, p, p, None, None, None) == -1
    assert Lv.ngp_rays_nonempty(p, 8, p, None, None, None, None) == -1
