"""CPU: the policy fixture and the test-side torch reference of the
notebooks' networks agree (so the GPU tests compare against the notebook's
own models), and the packed-parameter geometry the ABI reports."""
import numpy as np
import torch
from torch.distributions import Bernoulli

import golden_data as gd
from delivery_drone_amd import abi


def test_torch_reference_reproduces_notebook_models():
    d, nets = gd.policy_fixture()
    x = torch.from_numpy(d["obs"])
    with torch.no_grad():
        probs = gd.torch_mlp(nets["actor"])(x).numpy()
        values = gd.torch_mlp(nets["critic"])(x)[:, 0].numpy()
    np.testing.assert_array_equal(probs, d["probs"])
    np.testing.assert_array_equal(values, d["values"])
    assert d["obs"].shape[0] % 32 != 0  # a ragged last tile is exercised


def test_log_prob_fixture_is_bernoulli_sum():
    d, _ = gd.policy_fixture()
    lp = Bernoulli(probs=torch.from_numpy(d["probs"])).log_prob(torch.from_numpy(d["actions"])).sum(1)
    np.testing.assert_array_equal(lp.numpy(), d["log_prob"])


def test_packed_size_and_exports():
    lib = abi.lib()
    # A operands 2048 + 16384 + 8192, vectors 3*(128+128+64), last layer 192, bias + eps 4
    assert lib.dd_mlp_packed_floats() == 2048 + 16384 + 8192 + 960 + 192 + 4 + 4  # ... bias+eps, layout tag
    for name in ("dd_mlp_pack", "dd_mlp_forward"):
        assert hasattr(lib, name)


def test_forward_argument_errors_without_gpu():
    lib = abi.lib()
    io = abi.DDMlpIO()
    import ctypes
    for mode in (abi.DD_MLP_F32, abi.DD_MLP_F16X3):
        assert lib.dd_mlp_forward(None, mode, 2, ctypes.byref(io), 10, None) == 1   # bad out_dim
        assert lib.dd_mlp_forward(None, mode, 3, ctypes.byref(io), -1, None) == 1   # bad n
        assert lib.dd_mlp_forward(None, mode, 3, ctypes.byref(io), 0, None) == 0    # empty batch
        assert lib.dd_mlp_forward(None, mode, 3, ctypes.byref(io), 5, None) == 1    # null buffers
        assert lib.dd_mlp_pack(None, mode, None, None) == 1
    assert lib.dd_mlp_forward(None, 2, 3, ctypes.byref(io), 0, None) == 1           # bad compute
    io.obs = 16
    assert lib.dd_mlp_forward(ctypes.c_void_p(0x1008), abi.DD_MLP_F16X3, 3, ctypes.byref(io), 5, None) == 1
    params = abi.DDMlpParams(*([16] * 14), 3, 1e-5)
    assert lib.dd_mlp_pack(ctypes.byref(params), abi.DD_MLP_F16X3, ctypes.c_void_p(0x1004), None) == 1
    assert lib.dd_mlp_pack(None, 7, None, None) == 1
