import sys, torch
sys.path.insert(0, "reinforcement-learning-101_amd"); sys.path.insert(0, ".")
from delivery_drone_amd import EnvConfig, VecDroneEnv
dev = torch.device("cuda", 0)
for prec in ("f64", "f32"):
    for cfg in (dict(platform_moving=True), dict(wind_enabled=True, wind_x=0.05, wind_y=-0.02), dict(auto_reset=False)):
        c = EnvConfig(randomize_drone=True, seed=14, **cfg)
        a = VecDroneEnv(777, device=dev, config=c, precision=prec); b = VecDroneEnv(777, device=dev, config=c, precision=prec)
        a.reset(); b.reset()
        acts = torch.randint(0, 8, (80, 777), device=dev, dtype=torch.uint8, generator=torch.Generator(device=dev).manual_seed(0))
        obs, rew, done = a.rollout(acts)
        bad = None
        for t in range(80):
            o, r, d, _ = b.step(acts[t])
            if not (torch.equal(obs[t], o) and torch.equal(rew[t], r) and torch.equal(done[t], d)):
                diff = (obs[t] != o)
                lanes = diff.any(1).nonzero().flatten()[:3].tolist()
                cols = diff.any(0).nonzero().flatten().tolist()
                bad = (t, lanes, cols, [(obs[t, l].tolist(), o[l].tolist()) for l in lanes[:1]], (rew[t] != r).sum().item(), (done[t] != d).sum().item())
                break
        print(prec, cfg, "OK" if bad is None else bad, flush=True)
