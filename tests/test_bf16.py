"""bf16 forward warp (no reference counterpart).

The reference's FW is float32-only (alt_cuda/fw.py:40-43) and its extension
dispatches float / double only (fw_cuda_kernel.cu:70).  The spec defined here:
bf16 obj / output, float32 flow and depth keys, the coordinate arithmetic of
fw.py:27-42.  The warp selects source values and never computes with them, so
the parity bar is bit-exact: the output's bit patterns are the winners' bf16
bit patterns, i.e. the CPU oracle's float32 output on obj.float() truncated
back to bf16 (exact, since every value came from a bf16), and the masks are
the oracle's.
"""
import numpy as np
import pytest
import torch

from oracle import oracle


def _bits_to_bf16(bits: np.ndarray) -> torch.Tensor:
    return torch.from_numpy(bits.astype(np.int16)).view(torch.bfloat16)


def _oracle_bf16(obj_bits, flow, depth):
    """Expected (output bits uint16, valid, collision) from the float32 oracle."""
    obj32 = (obj_bits.astype(np.uint32) << 16).view(np.float32)
    out, valid, coll = oracle.fw_flow(obj32, flow, depth)
    return (np.ascontiguousarray(out).view(np.uint32) >> 16).astype(np.uint16), valid, coll


def _case(B, C, H, W, seed, scale=6.0):
    rng = np.random.default_rng(seed)
    # every bf16 bit pattern is a value the warp must move untouched (NaN payloads,
    # infinities, subnormals, -0) -- nothing is converted on the way
    obj_bits = rng.integers(0, 1 << 16, size=(B, C, H, W), dtype=np.uint16)
    flow = (rng.standard_normal((B, 2, H, W)) * scale).astype(np.float32)
    depth = np.round(rng.uniform(1, 20, (B, 1, H, W))).astype(np.float32)  # tie-heavy
    depth[rng.random(depth.shape) < 0.03] = 1000.0                          # collision path
    return obj_bits, flow, depth


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(2, 6, 48, 64), (1, 3, 37, 53), (3, 1, 16, 20), (2, 9, 24, 40),
                                   (1, 4, 1, 7), (2, 2, 5, 1)])
def test_bf16_warp_bit_exact_vs_oracle(shape):
    from opticalflowfromdepth_amd import forward_warp_flow
    B, C, H, W = shape
    obj_bits, flow, depth = _case(B, C, H, W, seed=sum(shape))
    dev = torch.device("cuda:0")
    obj = _bits_to_bf16(obj_bits).to(dev)
    out, valid, coll = forward_warp_flow(obj, torch.from_numpy(flow).to(dev), torch.from_numpy(depth).to(dev))
    assert out.dtype == torch.bfloat16 and valid.dtype == torch.float32
    e_out, e_valid, e_coll = _oracle_bf16(obj_bits, flow, depth)
    got_bits = out.cpu().view(torch.int16).numpy().view(np.uint16)
    assert np.array_equal(got_bits, e_out)
    assert np.array_equal(valid.cpu().numpy(), e_valid)
    assert np.array_equal(coll.cpu().numpy(), e_coll)


@pytest.mark.gpu
def test_bf16_warp_equals_f32_path_at_config5():
    """368x560 (config 5), disparity and ego-motion flows: the bf16 warp equals
    the float32 warp of the same values rounded to bf16, and its masks equal."""
    from opticalflowfromdepth_amd import forward_warp_flow, synth
    dev = torch.device("cuda:0")
    seeds = list(range(500, 508))
    obj, flow, depth = synth.stage_one_batch(seeds, 368, 560, dev)
    objb = obj.to(torch.bfloat16)
    got = forward_warp_flow(objb, flow, depth)
    ref = forward_warp_flow(objb.float(), flow, depth)
    assert torch.equal(got[0].view(torch.int16), ref[0].to(torch.bfloat16).view(torch.int16))
    assert torch.equal(got[1], ref[1]) and torch.equal(got[2], ref[2])


@pytest.mark.gpu
@pytest.mark.parametrize("short_tiles", [1, 0], ids=["tiles128x16", "tiles128x32"])
def test_bf16_warp_config5_batch_bit_exact_vs_oracle(short_tiles):
    """A config-5 call (16 images of 368x560, C=6, every bf16 bit pattern;
    a short call: one SPLAT workgroup per tile) on both tile heights
    (ofd_fw_set_short_tiles): the oracle's bits."""
    from opticalflowfromdepth_amd import _native, forward_warp_flow
    obj_bits, flow, depth = _case(16, 6, 368, 560, seed=5)
    dev = torch.device("cuda:0")
    lib = _native.lib()
    prev = lib.ofd_fw_set_short_tiles(short_tiles)
    try:
        out, valid, coll = forward_warp_flow(_bits_to_bf16(obj_bits).to(dev), torch.from_numpy(flow).to(dev),
                                             torch.from_numpy(depth).to(dev))
        torch.cuda.synchronize()
    finally:
        lib.ofd_fw_set_short_tiles(prev)
    e_out, e_valid, e_coll = _oracle_bf16(obj_bits, flow, depth)
    assert np.array_equal(out.cpu().view(torch.int16).numpy().view(np.uint16), e_out)
    assert np.array_equal(valid.cpu().numpy(), e_valid) and np.array_equal(coll.cpu().numpy(), e_coll)


@pytest.mark.gpu
def test_bf16_warp_argument_errors():
    from opticalflowfromdepth_amd import forward_warp_flow
    dev = torch.device("cuda:0")
    obj = torch.zeros(1, 3, 8, 8, dtype=torch.bfloat16, device=dev)
    flow = torch.zeros(1, 2, 8, 8, device=dev)
    depth = torch.ones(1, 1, 8, 8, device=dev)
    with pytest.raises(RuntimeError, match="float32 flow"):
        forward_warp_flow(obj, flow.double(), depth)
    with pytest.raises(RuntimeError, match="float32 depth"):
        forward_warp_flow(obj, flow, depth.double())
    bad_out = (torch.empty(1, 3, 8, 8, device=dev), torch.empty(1, 1, 8, 8, device=dev),
               torch.empty(1, 1, 8, 8, device=dev))
    with pytest.raises(RuntimeError, match="bfloat16"):
        forward_warp_flow(obj, flow, depth, out=bad_out)


def test_oracle_bf16_expectation_is_a_bit_copy():
    """The expectation helper itself (CPU): a 0-flow warp with distinct depths is the identity."""
    obj_bits = np.arange(2 * 3 * 4 * 5, dtype=np.uint16).reshape(2, 3, 4, 5) * 331
    flow = np.zeros((2, 2, 4, 5), np.float32)
    depth = np.ones((2, 1, 4, 5), np.float32)
    out, valid, coll = _oracle_bf16(obj_bits, flow, depth)
    assert np.array_equal(out, obj_bits) and valid.all() and not coll.any()
