"""GPU: dd_mlp_forward (the notebooks' actor / critic on f32 MFMA, and the
opt-in f16x3 split-operand form) against the notebook models' own outputs
(tests/golden/policy.npz) and a torch fp32 reference, plus the Bernoulli
sampling contract.

Tolerances (float32 model, different summation order than torch's), the same
for both compute modes except the critic's values: probabilities |d| <= 2e-6;
values |d| <= 1e-4 + 2e-6 |v| (f16x3: 4e-4 + 8e-6 |v|, VALUE_TOL);
log-probabilities |d| <= 1e-5 * (1 + |lp|).  (f16x3 keeps ~22 bits per
product, f32 accumulation: a numpy emulation on the fixture puts its actor
probabilities within 5e-7 of float64, f32's within 4e-7:
tools/mlp_split_sim.py.)"""
import numpy as np
import pytest
import torch
from torch.distributions import Bernoulli

import golden_data as gd
from delivery_drone_amd import MlpNet, VecDroneEnv

pytestmark = pytest.mark.gpu


def close(got, want, rel, abs_):
    got, want = np.asarray(got, np.float64), np.asarray(want, np.float64)
    err = np.abs(got - want)
    bound = abs_ + rel * np.abs(want)
    assert np.all(err <= bound), f"max err {err.max():.3g} at {np.argmax(err - bound)}"


@pytest.fixture(scope="module")
def fixture():
    return gd.policy_fixture()


COMPUTE = ("f32", "f16x3")
# critic values: the notebook critic's outputs reach |v| ~ 850 through a
# Linear(64, 1) with large weights, which amplifies the hidden layers'
# relative error; f16x3 keeps ~22 bits per product against f32's 24, so its
# bound is 4x f32's (emulation: 2.0e-4 vs 1.3e-4 from float64 at worst).
VALUE_TOL = {"f32": (2e-6, 1e-4), "f16x3": (8e-6, 4e-4)}


@pytest.mark.parametrize("compute", COMPUTE)
def test_actor_probs_match_notebook_model(fixture, gpu_device, compute):
    d, nets = fixture
    actor = MlpNet(nets["actor"], device=gpu_device, compute=compute)
    probs = actor(torch.as_tensor(d["obs"], device=gpu_device))
    close(probs.cpu().numpy(), d["probs"], 0.0, 2e-6)


@pytest.mark.parametrize("compute", COMPUTE)
def test_critic_values_match_notebook_model(fixture, gpu_device, compute):
    d, nets = fixture
    critic = MlpNet(nets["critic"], device=gpu_device, compute=compute)
    assert critic.out_dim == 1
    v = critic(torch.as_tensor(d["obs"], device=gpu_device))
    rel, abs_ = VALUE_TOL[compute]
    close(v.cpu().numpy(), d["values"], rel, abs_)


@pytest.mark.parametrize("compute", COMPUTE)
def test_log_prob_of_sampled_actions(fixture, gpu_device, compute):
    d, nets = fixture
    actor = MlpNet(nets["actor"], device=gpu_device, compute=compute)
    obs = torch.as_tensor(d["obs"], device=gpu_device)
    actions, lp, probs = actor.act(obs, seed=3, step=17, probs=True)
    bits = torch.stack([(actions >> j) & 1 for j in range(3)], dim=1).float()
    want = Bernoulli(probs=probs).log_prob(bits).sum(1)
    close(lp.cpu().numpy(), want.cpu().numpy(), 1e-5, 1e-5)
    # and against the notebook model's probabilities directly
    want_nb = Bernoulli(probs=torch.as_tensor(d["probs"])).log_prob(bits.cpu()).sum(1)
    close(lp.cpu().numpy(), want_nb.numpy(), 1e-5, 2e-5)


def test_sampling_is_bernoulli(fixture, gpu_device):
    """Bit j of the action is set with probability p_j: 64 draws (steps) of
    every fixture row; z-scores of the per-bit totals."""
    d, nets = fixture
    actor = MlpNet(nets["actor"], device=gpu_device)
    obs = torch.as_tensor(d["obs"], device=gpu_device)
    p = actor(obs).double()
    hits = torch.zeros_like(p)
    draws = 64
    for s in range(draws):
        a, _ = actor.act(obs, seed=99, step=s)
        hits += torch.stack([((a >> j) & 1).double() for j in range(3)], dim=1)
    mean = (p * draws).sum(0)
    var = (p * (1 - p) * draws).sum(0)
    z = ((hits.sum(0) - mean) / var.sqrt()).cpu().numpy()
    assert np.all(np.abs(z) < 5.0), z


def test_samples_are_keyed_by_env_and_step(fixture, gpu_device):
    d, nets = fixture
    actor = MlpNet(nets["actor"], device=gpu_device)
    obs = torch.as_tensor(d["obs"], device=gpu_device)
    a, lp = actor.act(obs, seed=5, step=40)
    a2, lp2 = actor.act(obs, seed=5, step=40)
    assert torch.equal(a, a2) and torch.equal(lp, lp2)
    cut = 1000  # two shards with their global env ids draw what the full batch draws
    b0, _ = actor.act(obs[:cut], seed=5, step=40)
    b1, _ = actor.act(obs[cut:], seed=5, step=40, env_id_base=cut)
    assert torch.equal(torch.cat([b0, b1]), a)
    a3, _ = actor.act(obs, seed=5, step=41)
    assert not torch.equal(a, a3)


@pytest.mark.parametrize("compute", COMPUTE)
@pytest.mark.parametrize("n", [1, 31, 32, 33, 4097, 65_536 + 37])
def test_random_weights_vs_torch_fp32(n, gpu_device, compute):
    """Freshly initialised networks (torch's default init) at ragged and
    config-5 sizes against torch on the same device."""
    torch.manual_seed(n)
    for k in (3, 1):
        sd = _random_sd(k)
        ref = gd.torch_mlp({kk: v.numpy() for kk, v in sd.items()}, device=gpu_device)
        net = MlpNet(sd, device=gpu_device, compute=compute)
        obs = torch.randn(n, 15, device=gpu_device) * 2.0
        with torch.no_grad():
            want = ref(obs)
        got = net(obs)
        if k == 1:
            want = want[:, 0]
        close(got.cpu().numpy(), want.cpu().numpy(), 1e-4 if k == 1 else 0.0, 1e-5 if k == 3 else 1e-4)


def _random_sd(k):
    from torch import nn
    layers = [nn.Linear(15, 128), nn.LayerNorm(128), nn.ReLU(), nn.Linear(128, 128), nn.LayerNorm(128), nn.ReLU(),
              nn.Linear(128, 64), nn.LayerNorm(64), nn.ReLU(), nn.Linear(64, k)]
    net = nn.Sequential(*layers)
    with torch.no_grad():  # non-trivial LayerNorm affine parameters
        for i in (1, 4, 7):
            net[i].weight.uniform_(0.5, 1.5)
            net[i].bias.uniform_(-0.2, 0.2)
    return net.state_dict()


@pytest.mark.parametrize("compute", COMPUTE)
def test_policy_driven_rollout_matches_host_loop(fixture, gpu_device, compute):
    """obs -> dd_mlp_forward (sample) -> dd_step for 40 frames, all on the
    device, equals the same loop with actions copied through the host."""
    d, nets = fixture
    actor = MlpNet(nets["actor"], device=gpu_device, compute=compute)
    a_env = VecDroneEnv(2048, device=gpu_device, randomize_drone=True, auto_reset=True, seed=4)
    b_env = VecDroneEnv(2048, device=gpu_device, randomize_drone=True, auto_reset=True, seed=4)
    oa, ob = a_env.reset(), b_env.reset()
    for t in range(40):
        acts, _ = actor.act(oa, seed=8, step=t)
        oa, ra, da, _ = a_env.step(acts)
        host = actor.act(ob, seed=8, step=t)[0].cpu()
        ob, rb, db, _ = b_env.step(host.to(gpu_device))
        assert torch.equal(oa, ob) and torch.equal(ra, rb) and torch.equal(da, db)


def test_errors(fixture, gpu_device):
    d, nets = fixture
    critic = MlpNet(nets["critic"], device=gpu_device)
    with pytest.raises(ValueError):
        critic.act(torch.zeros(4, 15, device=gpu_device))
    with pytest.raises(ValueError):
        critic(torch.zeros(4, 14, device=gpu_device))
    bad = dict(nets["actor"])
    bad["3.weight"] = bad["3.weight"][:, :64]
    with pytest.raises(ValueError):
        MlpNet(bad, device=gpu_device)
    with pytest.raises(ValueError):
        MlpNet(nets["actor"], device=gpu_device, compute="bf16")


def test_f16x3_tracks_f32(fixture, gpu_device):
    """The two compute modes agree with each other on the notebook model and
    on observations far from the fixture's (|obs| up to ~40)."""
    d, nets = fixture
    a32 = MlpNet(nets["actor"], device=gpu_device)
    a16 = MlpNet(nets["actor"], device=gpu_device, compute="f16x3")
    torch.manual_seed(7)
    obs = torch.cat([torch.as_tensor(d["obs"], device=gpu_device),
                     torch.randn(4096, 15, device=gpu_device) * 10.0])
    close(a16(obs).cpu().numpy(), a32(obs).cpu().numpy(), 0.0, 3e-6)


def test_packed_layout_tag_poisons_mismatched_launches(fixture, gpu_device):
    # a buffer packed for one compute / K and run as another gives NaN, not
    # numbers from misread weights; the right pairing stays finite
    from delivery_drone_amd import abi
    import ctypes
    d, nets = fixture
    obs = torch.as_tensor(d["obs"], device=gpu_device)
    n = obs.shape[0]
    lib = abi.lib()
    for compute, other in (("f32", abi.DD_MLP_F16X3), ("f16x3", abi.DD_MLP_F32)):
        actor = MlpNet(nets["actor"], device=gpu_device, compute=compute)
        critic = MlpNet(nets["critic"], device=gpu_device, compute=compute)
        probs = torch.empty(n, 3, device=gpu_device)
        lp = torch.empty(n, device=gpu_device)
        io = abi.DDMlpIO(obs.data_ptr(), probs.data_ptr(), None, lp.data_ptr(), 0, 0, 0)
        abi.check(lib.dd_mlp_forward(actor.packed.data_ptr(), other, 3, ctypes.byref(io), n, None), "fwd")
        torch.cuda.synchronize()
        assert bool(torch.isnan(probs).all()) and bool(torch.isnan(lp).all())
        vals = torch.empty(n, device=gpu_device)
        io = abi.DDMlpIO(obs.data_ptr(), vals.data_ptr(), None, None, 0, 0, 0)
        abi.check(lib.dd_mlp_forward(actor.packed.data_ptr(), actor._mode, 1, ctypes.byref(io), n, None), "fwd")
        torch.cuda.synchronize()
        assert bool(torch.isnan(vals).all())  # an actor buffer run as a critic
        io = abi.DDMlpIO(obs.data_ptr(), vals.data_ptr(), None, None, 0, 0, 0)
        abi.check(lib.dd_mlp_forward(critic.packed.data_ptr(), critic._mode, 1, ctypes.byref(io), n, None), "fwd")
        torch.cuda.synchronize()
        assert bool(torch.isfinite(vals).all())
        # dd_policy_rollout with a critic's buffer: NaN log-probabilities
        env = VecDroneEnv(64, device=gpu_device, randomize_drone=True)
        env.reset()
        critic.out_dim = 3  # get past the wrapper's own check to reach the C ABI
        _, _, lp2, _, _ = env.policy_rollout(critic, 3)
        torch.cuda.synchronize()
        assert bool(torch.isnan(lp2).all())
        _, _, lp3, _, _ = env.policy_rollout(actor, 3)
        assert bool(torch.isfinite(lp3).all())


def test_f16x3_refuses_weights_beyond_f16_range(fixture, gpu_device):
    _, nets = fixture
    for key, value in (("3.weight", 3000.0), ("4.weight", 12.0)):  # a hidden weight; a LayerNorm weight (out > 128)
        sd = {k: np.array(v, copy=True) for k, v in nets["actor"].items()}
        sd[next(k for k in sd if k.endswith(key))].flat[0] = value
        with pytest.raises(ValueError, match="f16x3"):
            MlpNet(sd, device=gpu_device, compute="f16x3")
        MlpNet(sd, device=gpu_device, compute="f32")  # f32 takes them


@pytest.mark.parametrize("compute", COMPUTE)
@pytest.mark.parametrize("n", [33, 65_536 + 37])
def test_observations_at_any_offset(fixture, gpu_device, compute, n):
    """The forward reads each row with unaligned loads (dd_mlp_forward's
    prologue: two 16-byte loads per lane from column 0 or 7 of a 60-byte row).
    Rows that start 4 or 12 bytes into an allocation, with the last row at its
    very end, give the same bits as an aligned copy."""
    _, nets = fixture
    actor = MlpNet(nets["actor"], device=gpu_device, compute=compute)
    critic = MlpNet(nets["critic"], device=gpu_device, compute=compute)
    torch.manual_seed(n)
    for skip in (1, 3):
        flat = torch.randn(n * 15 + skip, device=gpu_device)
        obs = flat[skip:].view(n, 15)  # ends exactly at the allocation's last float
        assert obs.data_ptr() % 16 != 0
        ref = obs.clone()
        assert torch.equal(actor(obs), actor(ref)) and torch.equal(critic(obs), critic(ref))
        a, lp = actor.act(obs, seed=2, step=9)
        a2, lp2 = actor.act(ref, seed=2, step=9)
        assert torch.equal(a, a2) and torch.equal(lp, lp2)


@pytest.mark.parametrize("compute", COMPUTE)
@pytest.mark.parametrize("ln", ["zero_weight", "zero_all", "wide_range", "negative"])
def test_layernorm_parameters_at_the_edges(gpu_device, compute, ln):
    """The ReLU is no v_max: f32 scales each LayerNorm's output below 1 by a
    power of two taken from its weight and bias (act_scale) and clamps, f16x3
    splits the output with its ReLU (split_pair_relu).  LayerNorm weights all
    zero (the output is the bias), weight and bias all zero (scale 1, every
    activation 0), weights from 1e-3 to 10 in one layer, and negative weights,
    against torch fp32."""
    from torch import nn
    torch.manual_seed(11)
    for k in (3, 1):
        layers = [nn.Linear(15, 128), nn.LayerNorm(128), nn.ReLU(), nn.Linear(128, 128), nn.LayerNorm(128), nn.ReLU(),
                  nn.Linear(128, 64), nn.LayerNorm(64), nn.ReLU(), nn.Linear(64, k)]
        net = nn.Sequential(*layers)
        with torch.no_grad():
            for i in (1, 4, 7):
                w, b = net[i].weight, net[i].bias
                if ln == "zero_weight":
                    w.zero_()
                    b.uniform_(-0.5, 0.5)
                elif ln == "zero_all":
                    w.zero_()
                    b.zero_()
                elif ln == "wide_range":
                    w.copy_(torch.logspace(-3, 1, w.numel())[torch.randperm(w.numel())])
                    b.uniform_(-0.2, 0.2)
                else:
                    w.uniform_(-1.5, -0.5)
                    b.uniform_(-0.2, 0.2)
        sd = net.state_dict()
        ref = gd.torch_mlp({kk: v.numpy() for kk, v in sd.items()}, device=gpu_device)
        got_net = MlpNet(sd, device=gpu_device, compute=compute)
        obs = torch.randn(4097, 15, device=gpu_device) * 2.0
        with torch.no_grad():
            want = ref(obs)
        got = got_net(obs)
        if k == 1:
            want = want[:, 0]
        scale = float(want.abs().max()) + 1.0
        close(got.cpu().numpy(), want.cpu().numpy(), 1e-4 if k == 1 else 0.0,
              (1e-5 if k == 3 else 1e-4) * (scale if k == 1 else 1.0))


@pytest.mark.parametrize("compute", COMPUTE)
def test_confident_actor_tail_vs_torch_fp32(gpu_device, compute):
    """the Sigmoid is v_rcp(1 + v_exp(-z log2 e)), whose relative
    error grows with |z| (about |z| f32 ulps of p for z < 0).  A network whose
    logits sit near -14, -8 and +4 (probabilities ~8e-7, ~3e-4, ~1 - 0.018):
    probabilities against torch fp32 to a RELATIVE bound (f32 5e-5, f16x3 5e-4:
    it covers the logits' own difference from torch's summation order, dp/p =
    dz, plus the exp's ~|z| ulps), and the summed log-probability of sampled
    actions to 5e-5 (5e-4) x (1 + |lp|)."""
    torch.manual_seed(11)
    sd = _random_sd(3)
    sd["9.bias"] = torch.tensor([-14.0, -8.0, 4.0])
    sd["9.weight"] = sd["9.weight"] * 0.05  # logits dominated by the bias: deep in the tails
    ref = gd.torch_mlp({k: v.numpy() for k, v in sd.items()}, device=gpu_device)
    net = MlpNet(sd, device=gpu_device, compute=compute)
    obs = torch.randn(4096, 15, device=gpu_device)
    with torch.no_grad():
        want = ref(obs).double()
    got = net(obs).double()
    rel = 5e-5 if compute == "f32" else 5e-4
    assert float(want[:, 0].max()) < 1e-5 and float(want[:, 2].min()) > 0.95  # the tails are exercised
    err = ((got - want).abs() / want.clamp_min(1e-30))
    err[:, 2] = (got[:, 2] - want[:, 2]).abs() / (1 - want[:, 2]).clamp_min(1e-30)  # p ~ 1: relative in 1 - p
    assert float(err.max()) <= rel, f"max relative error {float(err.max()):.3g}"
    actions, lp, probs = net.act(obs, seed=3, step=1, probs=True)
    bits = torch.stack([(actions.long() >> j) & 1 for j in range(3)], 1).double()
    want_lp = Bernoulli(probs=want).log_prob(bits).sum(1)
    assert float(((lp.double() - want_lp).abs() / (1 + want_lp.abs())).max()) <= rel
