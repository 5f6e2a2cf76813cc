"""torch-tensor ops: the plain-PyTorch reference (CPU, bit-exact vs the oracle) and the HIP
kernels driven through torch tensors (GPU, bit-exact vs the PyTorch reference)."""
import numpy as np
import pytest
import torch

from heat2d_amd import ops
from heat2d_amd.ops import reference as R


@pytest.mark.parametrize("boundary", ["fixed", "ghost-zero"])
@pytest.mark.parametrize("per", [(False, False), (True, True)])
def test_torch_reference_bitexact_vs_oracle(native, boundary, per):
    nx, ny, steps = 31, 29, 25
    u = R.center_hot(nx, ny)
    got = R.run(u, steps, boundary=boundary, periodic=per).numpy()
    ref = native.oracle_run(nx, ny, steps, boundary=0 if boundary == "fixed" else 1, periodic_x=per[0],
                            periodic_y=per[1])["grid"]
    assert np.array_equal(got, ref)


def test_center_hot_matches_native(native):
    assert np.array_equal(R.center_hot(97, 130).numpy(), native.init_global(97, 130, 0))


def test_heat_steps_cpu_uses_oracle(native):
    u = R.center_hot(20, 30)
    assert torch.equal(ops.heat_steps(u, 17), R.run(u, 17))


def test_ops_refuse_cpu_tiles():
    g, t = ops.alloc_tile(16, 16, 4, device="cpu")
    with pytest.raises(ValueError):
        ops.stencil(t, t.clone(), g, 1)


@pytest.mark.gpu
@pytest.mark.parametrize("K", [1, 4, 8])
@pytest.mark.parametrize("boundary", ["fixed", "ghost-zero"])
def test_hip_stencil_vs_torch_reference(gpu, K, boundary):
    nx, ny = 200, 333
    g, a = ops.alloc_tile(nx, ny, 8, device="cuda")
    ops.init_tile(a, g)
    b = torch.zeros_like(a)
    ops.stencil(a, b, g, K, boundary=boundary)
    ref = R.run(R.center_hot(nx, ny, "cuda"), K, boundary=boundary)
    assert torch.equal(ops.owned(b, g), ref)


@pytest.mark.gpu
def test_hip_fp32_vs_torch_fp32_reference(gpu):
    nx, ny, steps = 180, 260, 40
    u = R.center_hot(nx, ny, "cuda")
    got = ops.heat_steps(u, steps, precision="fp32")
    ref = R.run(u, steps, precision="fp32")
    rel = ((got - ref).abs().max() / ref.abs().max()).item()
    assert rel < 2e-6, rel


@pytest.mark.gpu
@pytest.mark.parametrize("per", [(True, False), (False, True), (True, True)])
def test_heat_steps_periodic_gpu(gpu, per):
    nx, ny, steps = 64, 300, 19
    u = R.center_hot(nx, ny, "cuda")
    got = ops.heat_steps(u, steps, boundary="ghost-zero", periodic=per)
    assert torch.equal(got, R.run(u, steps, boundary="ghost-zero", periodic=per))


@pytest.mark.gpu
def test_naive_op_and_residual(native, gpu):
    nx, ny = 100, 140
    g, a = ops.alloc_tile(nx, ny, 4, device="cuda")
    ops.init_tile(a, g)
    b = torch.zeros_like(a)
    ops.naive_step(a, b, g)
    ref = R.step(R.center_hot(nx, ny, "cuda"))
    assert torch.equal(ops.owned(b, g), ref)
    part = torch.zeros(4096, dtype=torch.float64, device="cuda")
    c = torch.zeros_like(a)
    ops.stencil(a, c, g, 1, residual=part)
    expect = ((ref.double() - R.center_hot(nx, ny, "cuda").double()) ** 2).sum().item()
    assert abs(part.sum().item() - expect) / expect < 1e-12
