import sys; sys.path.insert(0, 'tests'); sys.path.insert(0, '.'); sys.path.insert(0, 'reinforcement-learning-101_amd')
import numpy as np, torch
import golden_data as gd
from delivery_drone_amd import VecDroneEnv, EnvConfig
r = gd.npz('single_step.npz'); e = gd.expected_outputs(r)
for prec in ("f32", "f64"):
    n = r['in_x'].shape[0]
    env = VecDroneEnv(n, precision=prec, device='cuda:0')
    for k, v in gd.state_from_inputs(r).items():
        t = getattr(env, k); t.copy_(torch.as_tensor(v, dtype=t.dtype))
    obs, rew, done, info = env.step(torch.as_tensor(r['in_action'], device='cuda:0'))
    torch.cuda.synchronize()
    rew = rew.cpu().numpy().astype(np.float64); tot = env.total_reward.cpu().numpy().astype(np.float64)
    bad = np.flatnonzero(np.abs(rew - e['reward']) > 1e-5)
    print(prec, 'reward mismatches', len(bad))
    for i in bad[:8]:
        print('  ', i, 'gpu', rew[i], 'ref', e['reward'][i], 'tot gpu', tot[i], 'ref', e['total_reward'][i], 'x', e['x'][i], 'y', e['y'][i], 'fuel', e['fuel'][i])
    badt = np.flatnonzero(np.abs(tot - e['total_reward']) > 1e-4)
    print(prec, 'total mismatches', len(badt))
    for i in badt[:8]:
        print('  ', i, 'tot gpu', tot[i], 'ref', e['total_reward'][i], 'in', r['in_total'][i], 'rew gpu', rew[i])
