#!/usr/bin/env python
"""Headline benchmark: MOPO model-rollout transitions/s on halfcheetah-mixed (BASELINE.json).

Workload (BASELINE.json configs[1]; examples/config/d4rl/halfcheetah_mixed.py + base.py + base_mopo.py):
  obs 17, act 6, ensemble 7 (5 elites), hidden 200, separate mean/var heads, learned-var penalty
  coeff 1.0, rollout_batch 50,000 per GPU, horizon 5, fp32, policy 256-256, model pool 1.25M rows
  (mopo.py:693-695).  One step = one ``MOPO._rollout_model`` (mopo.py:723-765): start-state gather
  from a 101,000-row env pool, 5 x (actor -> ensemble -> FakeEnv post -> pool append).
  Synthetic data / random-init weights (D4RL and pretrained .mat weights are not available offline).

Multi-GPU (torchrun, one rank per GPU, RCCL): weak scaling -- every rank rolls out its own 50,000
rows (disjoint Philox sub-streams) into a staging buffer; an all-gather over xGMI then appends all
ranks' transitions, in global row order, to every rank's replicated device pool; the timed region
includes the all-gather.  value = all ranks' transitions / max-over-ranks time.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from mopo_amd.bnn import DEFAULT_ENSEMBLE_DTYPE, DTYPES  # noqa: E402  (no torch / HIP import at this point)

O, A, E, ELITES, H, HP = 17, 6, 7, 5, 200, 256
ENV_ROWS = 101000
FLOP_BNN_ROW = 2 * E * ((O + A) * H + 3 * H * H + 2 * H * (O + 1))       # 1,845,200
FLOP_ACTOR_ROW = 2 * (O * HP + HP * HP + HP * 2 * A)                      # 145,920
PMC_SUMMARY = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'profiles', 'r06_pmc_summary.json')
MFMA_F32_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md: FP32 matrix (f32-in MFMA) dense peak
# ensemble dtype -> (bf16 parts per operand, bf16 products per f32 product); fp32 runs f32 MFMA
SPLIT = {'bf16': (1, 1), 'bf16x3': (2, 3), 'bf16x6': (3, 6), 'f16x3': (2, 3)}
DTYPE_DESC = {'fp32': 'fp32 (f32 MFMA 16x16x4)',
              'bf16x6': 'f32 (exact f32 operands: each split into 3 round-to-nearest bf16 parts with x0+x1+x2 == x '
                        'for 2^-100 <= |x| < 2^127; 6 bf16 MFMA products, the 3 dropped ones <= 2^-23 |x w| in total; '
                        'f32 accumulate; held to the fp32 parity tolerances)',
              'bf16x3': 'f32 operands as 2 bf16 parts (3 bf16 MFMA products, ~17 significand bits, f32 accumulate)',
              'bf16': 'bf16 (f32 accumulate)',
              'f16x3': 'f32 (f32 operands as 2 fp16 parts under power-of-two scales, 3 f16 MFMA products, f32 '
                       'accumulate: ~22-bit operands like bf16x6, held to the fp32 parity tolerances)'}


def dtype_desc(ensemble_dtype, actor_dtype=None):
    """The line's dtype: the ensemble forward's arithmetic and the rollout actor's (rollout.default_actor_dtype)."""
    from mopo_amd.rollout import default_actor_dtype
    act = actor_dtype or default_actor_dtype(ensemble_dtype)
    return '%s; rollout actor: %s' % (DTYPE_DESC[ensemble_dtype], {'fp32': 'exact f32 MFMA', 'bf16x6': 'the same exact '
                                      'bf16x6 split'}.get(act, 'f16x3 (~22-bit operands)'))


# BASELINE.json configs.  B_total = the config's rollout_batch; 'sharded': the batch is
# split over the ranks (C4, C5: 400k / 1M over 8 GPUs), otherwise every GPU runs B_total rows (weak scaling).
CONFIGS = {
    'C2': dict(name='halfcheetah-mixed (examples.config.d4rl.halfcheetah_mixed)', E=7, H=200, B_total=50000, h=5,
               domain='halfcheetah', penalty=1.0, env_rows=101000),
    'C3': dict(name='walker2d-medium-replay, bf16 ensemble', E=7, H=200, B_total=100000, h=1, domain='walker2d',
               penalty=1.0, env_rows=101000, dtype='bf16'),
    'C4': dict(name='halfcheetah-medium-expert, 400k rows sharded over the GPUs', E=7, H=200, B_total=400000, h=5,
               domain='halfcheetah', penalty=5.0, env_rows=1000000, sharded=True),
    'C5': dict(name='halfcheetah-mixed stress, E=32, H=400, 1M rows sharded over the GPUs', E=32, H=400,
               B_total=1000000, h=5, domain='halfcheetah', penalty=1.0, env_rows=101000, sharded=True),
    # BASELINE.json north_star's target workload: halfcheetah-mixed at rollout_batch=100k, horizon 5
    'N2': dict(name='halfcheetah-mixed north-star target, rollout_batch=100k, horizon 5', E=7, H=200,
               B_total=100000, h=5, domain='halfcheetah', penalty=1.0, env_rows=101000),
}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument('--gpus', type=int, default=1)
    p.add_argument('--steps', type=int, default=20)
    p.add_argument('--warmup', type=int, default=10, help='untimed rollouts first (the clocks ramp up over ~20 ms)')
    p.add_argument('--batch', type=int, default=50000)
    p.add_argument('--horizon', type=int, default=5)
    p.add_argument('--no-cpu-baseline', action='store_true')
    p.add_argument('--cpu-batch', type=int, default=10000,
                   help='rows of the C2 CPU-baseline rollout sample (the headline workload at fewer rows, labelled '
                        'as a sample in the bench line; each of the 6 runs takes a few seconds; 50000 = the whole '
                        'config, about a minute)')
    p.add_argument('--sac-steps', type=int, default=1000)
    p.add_argument('--cpu-sac-steps', type=int, default=1000)
    p.add_argument('--no-c3', action='store_true', help='skip the secondary C3 (bf16 walker2d) line')
    p.add_argument('--train-epochs', type=int, default=6,
                   help='timed BNN.train epochs in one train() call (0: skip); 6 is the fewest a from-scratch MOPO '
                        'model-training call runs (mopo.py:528 passes max_epochs=None, bnn.py:326 stops only after '
                        'more than max_epochs_since_update=5 epochs without improvement); the per-call draws, '
                        'holdout evaluation and repack are inside the timed region')
    p.add_argument('--cpu-train-steps', type=int, default=10)
    p.add_argument('--ensemble-dtype', default=DEFAULT_ENSEMBLE_DTYPE, choices=list(DTYPES),
                   help='headline ensemble-forward arithmetic (mopo_amd.bnn.DTYPES); the default is the one '
                        'MOPO.train runs (mopo_amd.bnn.DEFAULT_ENSEMBLE_DTYPE)')
    p.add_argument('--actor-dtype', default=None, choices=['fp32', 'bf16x6', 'f16x3'],
                   help="the rollout policy's arithmetic (default: mopo_amd.rollout.default_actor_dtype of the "
                        'ensemble dtype)')
    p.add_argument('--no-alt-dtypes', action='store_true',
                   help='skip the extra headline-workload lines with the other ensemble dtypes')
    p.add_argument('--prof-steps', type=int, default=20, help='untimed rollouts timed per kernel with HIP events')
    p.add_argument('--config', default='C2', choices=sorted(CONFIGS),
                   help='BASELINE.json workload of the main line (C2 = the headline); the per-rank batch is the '
                        "config's total rollout_batch / world for C4 / C5")
    p.add_argument('--shards', type=int, default=None,
                   help='sharded configs (C4, C5): split the batch over this many GPUs (default: the world size); '
                        '--shards 8 on one GPU runs one GPU\'s share of the 8-GPU config')
    a = p.parse_args()
    spec = CONFIGS[a.config]
    if a.config != 'C2':   # the config fixes the workload; --batch / --horizon apply to C2 only
        world = int(os.environ.get('WORLD_SIZE', '1'))
        a.batch = spec['B_total'] // (a.shards or world) if spec.get('sharded') else spec['B_total']
        a.horizon = spec['h']
        if a.ensemble_dtype == DEFAULT_ENSEMBLE_DTYPE and spec.get('dtype'):
            a.ensemble_dtype = spec['dtype']
        elif a.ensemble_dtype == DEFAULT_ENSEMBLE_DTYPE:   # the product default at this width (bf16x6: H <= 256)
            from mopo_amd.bnn import default_ensemble_dtype
            a.ensemble_dtype = default_ensemble_dtype(spec['H'])
    return a


def dist_setup(args):
    import torch
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if world > 1:
        import torch.distributed as dist
        # one rank per GPU; MOPO_DIST_BACKEND=gloo + wrapping devices is for rehearsing the
        # collective path with several ranks on one GPU (the driver's runs use RCCL)
        backend = os.environ.get('MOPO_DIST_BACKEND', 'nccl')
        dev_i = local % max(torch.cuda.device_count(), 1)
        torch.cuda.set_device(dev_i)
        if backend == 'nccl':
            dist.init_process_group('nccl', device_id=torch.device('cuda', dev_i))
        else:
            dist.init_process_group(backend)
        return rank, world, torch.device('cuda', dev_i)
    torch.cuda.set_device(0)
    return rank, world, torch.device('cuda', 0)


def spec_flop_row(spec):
    return 2 * spec['E'] * ((O + A) * spec['H'] + 3 * spec['H'] ** 2 + 2 * spec['H'] * (O + 1))


def make_env(spec, seed=0):
    """Synthetic env pool of the config's size: obs ~ N(0, 1), actions ~ U(-1, 1); walker2d
    heights / angles spread over the termination bounds so rows terminate at a moderate rate."""
    rs = np.random.RandomState(seed)
    n = spec['env_rows']
    env_obs = rs.normal(size=(n, O)).astype(np.float32)
    if spec['domain'] == 'walker2d':
        env_obs[:, 0] = rs.uniform(0.7, 2.1, n)
        env_obs[:, 1] = rs.uniform(-1.1, 1.1, n)
    env_act = rs.uniform(-1, 1, size=(n, A)).astype(np.float32)
    return env_obs, env_act


def build(args, dev, rank, world=None):
    import torch
    from mopo_amd.bnn import construct_model
    from mopo_amd.replay_pool import SimpleReplayPool
    from mopo_amd.rollout import ModelRollout, init_sac_params
    spec = CONFIGS[args.config]
    env_obs, env_act = make_env(spec)   # identical on every rank (replicated D4RL data)
    model = construct_model(obs_dim=O, act_dim=A, hidden_dim=spec['H'], num_networks=spec['E'], num_elites=ELITES,
                            separate_mean_var=True, seed=1, dtype=args.ensemble_dtype)
    mats = model.get_params()
    x = np.concatenate([env_obs, env_act], 1)
    mats[0] = x.mean(0, keepdims=True).astype(np.float32)                 # scaler.fit (utils.py:79-81)
    mats[1] = x.std(0, keepdims=True).astype(np.float32)
    model.set_params(mats)
    model.set_elites([0, 1, 2, 3, 4])
    world = int(os.environ.get('WORLD_SIZE', '1')) if world is None else world
    pool_rows = 5 * args.horizon * args.batch * world                       # mopo.py:693-695 (x ranks)
    pool = SimpleReplayPool(obs_dim=O, act_dim=A, max_size=pool_rows)
    pi = torch.from_numpy(init_sac_params(O, A, HP, seed=2)).to(dev)
    env = torch.from_numpy(env_obs).to(dev)
    staging = None
    if world > 1:  # per-step staging blocks gathered while the next step computes
        from mopo_amd.distributed import DistributedRollout
        staging = DistributedRollout(model, args.batch, args.horizon, O, A, device=dev)
        ro = staging.ro
    else:
        ro = ModelRollout(model, args.batch, args.horizon)
    return model, pool, ro, pi, env, staging


def rollout_step(args, ro, pool, pi, env, staging, epoch, rank, world):
    """One MOPO._rollout_model; returns transitions added (device tensor)."""
    from mopo_amd.static import static_fns
    spec = CONFIGS[args.config]
    tk, pen = static_fns[spec['domain']].term_kind, spec['penalty']
    if world == 1:
        return ro.run(env, pi, pool, args.batch, args.horizon, tk, pen, [0, 1, 2, 3, 4], seed=88, epoch=epoch,
                      actor_dtype=getattr(args, 'actor_dtype', None))
    # RCCL all-gather of each step's staged transitions (overlapping the next step) into every rank's pool
    return staging.run(env, pi, pool, tk, pen, [0, 1, 2, 3, 4], seed=88, epoch=epoch)


def blas_threads():
    """Threads the numpy oracle actually runs on (the BLAS pool; 1 if it cannot be read)."""
    try:
        from threadpoolctl import threadpool_info
        return int(max([i.get('num_threads', 1) for i in threadpool_info() if i.get('user_api') == 'blas'] or [1]))
    except Exception:
        return 1


CPU_RUNS = 5   # the median of >= 5 runs after 1 warm-up, fixed seeds


def median_runs(fn, runs=CPU_RUNS):
    """One warm-up call, then ``runs`` timed calls of ``fn() -> (units, seconds)``; returns the median rate,
    the per-run rates and the total sample."""
    fn()
    rates, units, secs = [], 0, 0.0
    for _ in range(runs):
        u, dt = fn()
        rates.append(u / dt)
        units += u
        secs += dt
    return float(np.median(rates)), [float(r) for r in rates], units, secs


def cpu_rollout_leg(B, horizon, domain='halfcheetah', penalty=1.0, env_rows=20000, seed=0):
    """The oracle's ``_rollout_model`` (numpy port of mopo.py:723-765 with the fp32 ensemble, FakeEnv and
    the static termination fns): start-state gather through the final pool append, fixed seed per run."""
    from oracle import bnn as obnn
    from oracle import fake_env as ofe
    from oracle import replay_pool as opool
    from oracle import rollout as orollout
    from oracle import sac as osac
    rs = np.random.RandomState(seed)
    env_obs = rs.normal(size=(env_rows, O)).astype(np.float32)
    if domain == 'walker2d':
        env_obs[:, 0] = rs.uniform(0.9, 1.9, env_rows)
        env_obs[:, 1] = rs.uniform(-0.9, 0.9, env_rows)
    fit = min(env_rows, 20000)
    p = obnn.init_params(E, O, A, hidden=H, seed=1, inputs=np.concatenate([env_obs[:fit], rs.uniform(-1, 1, (fit, A))], 1))
    P = osac.init_params(O, A, HP, seed=2)[:8]
    envp = opool.Pool(O, A, env_rows)
    envp.add_samples({'observations': env_obs, 'actions': np.zeros((env_rows, A)), 'rewards': np.zeros((env_rows, 1)),
                      'terminals': np.zeros((env_rows, 1), bool), 'next_observations': env_obs})

    def run():
        mp = opool.Pool(O, A, B * horizon)
        np.random.seed(88)
        t0 = time.perf_counter()
        out = orollout.rollout(envp, mp, p, [0, 1, 2, 3, 4], P, B, horizon, ofe.TERMINATION[domain], penalty,
                               eps_act=lambda n: np.random.normal(size=(n, A)))
        return sum(out['steps_added']), time.perf_counter() - t0
    return run


def cpu_baseline(args):
    """The CPU baseline of BASELINE.md section 3: the numpy restatement of the reference rollout (fp32
    ensemble; the reference's own TF path cannot run here), BLAS on the host's cores, the median of 5 runs
    after a warm-up, on bounded samples of each BASELINE config's workload (same E, H, horizon, domain,
    penalty and env-pool size; fewer rows, so the default bench stays within minutes)."""
    threads = blas_threads()
    legs = {}
    # (config, sample rows, horizon, domain, penalty, env rows, config description, the config's own rows)
    for key, B, h, dom, pen, env_rows, what, full in (
            ('C1', 1000, 1, 'halfcheetah', 1.0, 20000, 'halfcheetah_mixed plumbing config, h=1', 1000),
            ('C2', args.cpu_batch, args.horizon, 'halfcheetah', 1.0, 20000, 'halfcheetah-mixed, h=5', 50000),
            ('C3', 20000, 1, 'walker2d', 1.0, 20000, 'walker2d-medium-replay, h=1 (fp32 on CPU)', 100000),
            ('C4', 5000, 5, 'halfcheetah', 5.0, 1000000, 'halfcheetah-medium-expert, penalty 5, 1e6-row env pool, h=5',
             400000)):
        med, runs, units, secs = median_runs(cpu_rollout_leg(B, h, dom, pen, env_rows))
        scope = 'the whole config' if B == full else 'a sample of %d rollout rows (the config runs %d)' % (B, full)
        legs[key] = {'value': med, 'unit': 'transitions/s', 'runs': runs, 'median': med, 'cores': int(threads),
                     'rows_sampled': B, 'rows_config': full,
                     'sample': '%s, E=%d, H=%d: %s; %d timed runs (%d transitions in %.2f s) after 1 warm-up'
                               % (what, E, H, scope, CPU_RUNS, units, secs)}
    c2 = legs['C2']
    return {'value': c2['median'], 'unit': 'transitions/s', 'cores': int(threads), 'kind': 'port',
            'runs': c2['runs'], 'median': c2['median'],
            'rows_sampled': c2['rows_sampled'], 'rows_config': c2['rows_config'],
            'sample': 'oracle numpy rollout (mopo.py:723-765 restated), ' + c2['sample'], 'configs': legs}


def cpu_baseline_1core(args):
    """The same oracle rollout with BLAS limited to one thread (the C2 workload on a smaller sample)."""
    try:
        from threadpoolctl import threadpool_limits
    except Exception:
        return None
    with threadpool_limits(limits=1):
        med, runs, units, secs = median_runs(cpu_rollout_leg(3000, args.horizon))
    return {'value': med, 'unit': 'transitions/s', 'cores': 1, 'kind': 'port', 'runs': runs, 'median': med,
            'sample': 'oracle numpy rollout, 1 BLAS thread, B=3000, h=%d, E=%d, H=%d: %d timed runs (%d transitions '
                      'in %.2f s) after 1 warm-up' % (args.horizon, E, H, CPU_RUNS, units, secs)}


BF16_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: BF16 dense MFMA


def ensemble_bytes(rows, spec, dtype):
    """Algorithmic HBM bytes of one rollout-mode ensemble launch: the scaled input
    rows (32 f32 slots each), the weights once (f32, or the 16-bit parts), and per row the selected
    member's mean / std (2 x 18 f32), the penalty bits and the member index."""
    E, H, IN, D = spec['E'], spec['H'], O + A, O + 1
    n_w = E * (IN * H + 3 * H * H + 2 * H * D)
    wbytes = 4 * n_w if dtype == 'fp32' else 2 * SPLIT[dtype][0] * n_w
    return rows * (32 * 4 + 2 * D * 4 + 4 + 4) + wbytes


def roofline_of(dtype, rows, ms, flop_row=FLOP_BNN_ROW, hidden=200):
    """Roofline of the ensemble-forward launch: f32 MFMA for fp32; executed bf16 MFMA flops (products x
    the algorithmic f32 flops) against the bf16 dense peak for the split / bf16 kernels.  ``hidden`` picks the
    kernel name the library dispatches at that width (csrc/bnn.hip launch_bnn_fwd: the ring at H <= 256)."""
    alg = rows * flop_row / (ms * 1e-3) / 1e12
    wide = hidden > 256
    if dtype == 'fp32':
        return {'bound': 'mfma', 'kernel': 'bnn_fwd_kernel (ensemble forward, f32 MFMA 16x16x4)',
                'achieved': alg, 'peak': MFMA_F32_PEAK_TFLOPS, 'unit': 'TFLOP/s', 'frac': alg / MFMA_F32_PEAK_TFLOPS,
                'flop_per_launch': rows * flop_row, 'avg_launch_ms': ms}
    parts, prods = SPLIT[dtype]
    if dtype == 'f16x3' and wide:
        kern = ('bnn_fwd_f16h_kernel (ensemble forward in column halves, f16 MFMA 16x16x32, 3 products per f32 '
                'product)')
    elif dtype == 'f16x3':
        kern = ('bnn_fwd_ring_kernel<P=2> (ensemble forward on a 3-slot LDS ring, f16 MFMA 16x16x32, 3 products per f32 '
                'product)')
    elif dtype == 'bf16x6' and not wide:
        kern = ('bnn_fwd_ring_kernel<P=3> (ensemble forward on a 3-slot LDS ring, exact 3-part bf16 split, bf16 MFMA '
                '16x16x32, 6 products per f32 product)')
    else:
        kern = 'bnn_fwd_bf16_kernel<P=%d> (ensemble forward, bf16 MFMA 16x16x32, %d products per f32 product)' % (
            parts, prods)
    return {'bound': 'mfma', 'kernel': kern,
            'achieved': alg * prods, 'peak': BF16_PEAK_TFLOPS, 'unit': 'TFLOP/s',
            'frac': alg * prods / BF16_PEAK_TFLOPS, 'achieved_note': 'executed 16-bit MFMA TFLOP/s = %d x the '
            'algorithmic f32 rate (bf16 and f16 share the 2.5 PF dense peak)' % prods, 'algorithmic_f32_tflops': alg,
            'flop_per_launch': rows * flop_row, 'bf16_flop_per_launch': prods * rows * flop_row,
            'avg_launch_ms': ms}


KERNEL_CLASSES = ['start', 'actor', 'ensemble_fwd', 'fakeenv_post', 'compact', 'advance']


def kernel_profile(args, ro, pool, pi, env, staging, epoch0, rank, world, n):
    """Per-kernel-class average launch ms from ``n`` extra, untimed rollouts with HIP events on the
    rollout's own streams around every launch (mopo_rollout_profile; the records would add gaps to a
    timed region, so they never run inside one)."""
    import torch
    from mopo_amd import _lib as L
    L.check(L.lib().mopo_rollout_profile(ro._h, 1))
    for s in range(n):
        rollout_step(args, ro, pool, pi, env, staging, epoch0 + s, rank, world)
    torch.cuda.synchronize()
    ms = (C_double * 6)()
    nl = (C_int64 * 6)()
    L.check(L.lib().mopo_rollout_profile_read(ro._h, ms, nl, 6))
    L.check(L.lib().mopo_rollout_profile(ro._h, 0))
    return {k: ms[i] / max(nl[i], 1) for i, k in enumerate(KERNEL_CLASSES)}, {k: int(nl[i]) for i, k in
                                                                              enumerate(KERNEL_CLASSES)}


def leg_roofline(args, kms):
    """The roofline object of one leg: the ensemble launch (every launch processes args.batch rows on
    these workloads: halfcheetah never terminates, walker2d legs have horizon 1) priced per dtype, with
    the PMC HBM bytes of the same workload when they were collected."""
    spec = CONFIGS[args.config]
    r = roofline_of(args.ensemble_dtype, args.batch, kms['ensemble_fwd'], spec_flop_row(spec), spec['H'])
    r['traffic'] = pmc_traffic(args)
    r['traffic_note'] = ('HBM bytes per launch: 2 x FETCH_SIZE + WRITE_SIZE (gfx950 correction, MI355X_MICROARCH.md '
                         'HBM) from the committed --pmc passes of this workload, ' + os.path.relpath(PMC_SUMMARY, ROOT)
                         if r['traffic'] is not None else 'no PMC pass committed for this workload')
    r['algorithmic_bytes_per_launch'] = ensemble_bytes(args.batch, spec, args.ensemble_dtype)
    return r


def timed_leg(a2, dev, reps, warm, prof):
    """Build a2's workload on one rank, time ``reps`` back-to-back rollouts, then profile ``prof`` more."""
    import torch
    _, pool, ro, pi, env, _ = build(a2, dev, 0, world=1)
    for w in range(warm):
        rollout_step(a2, ro, pool, pi, env, None, w, 0, 1)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    st = [rollout_step(a2, ro, pool, pi, env, None, warm + i, 0, 1) for i in range(reps)]
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    n = int(sum(int(x.sum().item()) for x in st))
    kms, nl = kernel_profile(a2, ro, pool, pi, env, None, warm + reps, 0, 1, prof)
    return n, dt, kms


def alt_headline_leg(args, dev, dtype, reps=10):
    """The headline workload (same synthetic model / env pool / seeds as build()) with another ensemble
    dtype; one rank, rollouts timed back to back like the headline, then profiled for its roofline."""
    a2 = argparse.Namespace(**vars(args))
    a2.ensemble_dtype = dtype
    n, dt, kms = timed_leg(a2, dev, reps, 2, max(args.prof_steps // 2, 4))
    return {'metric': 'model-rollout transitions/s (halfcheetah-mixed, %s ensemble)' % dtype, 'value': n / dt,
            'unit': 'transitions/s', 'dtype': dtype_desc(dtype), 'ms_per_rollout': dt / reps * 1e3,
            'kernel_ms_avg': kms, 'roofline': leg_roofline(a2, kms)}


def config_leg(args, dev, name, dtype, reps=5, warm=3):
    """Another BASELINE config on this GPU (one rank's share of a sharded config): same synthetic
    construction and timing as the main line, then profiled for its roofline."""
    spec = CONFIGS[name]
    a2 = argparse.Namespace(**vars(args))
    a2.config, a2.ensemble_dtype, a2.horizon = name, dtype, spec['h']
    a2.batch = spec['B_total'] // 8 if spec.get('sharded') else spec['B_total']
    n, dt, kms = timed_leg(a2, dev, reps, warm, max(args.prof_steps // 4, 3))
    fr = spec_flop_row(spec)
    v = n / dt
    share = ' (one GPU of eight: %d of %d rows)' % (a2.batch, spec['B_total']) if spec.get('sharded') else ''
    out = {'metric': 'model-rollout transitions/s (%s: %s%s)' % (name, spec['name'], share), 'value': v,
           'unit': 'transitions/s', 'dtype': dtype_desc(dtype), 'ms_per_rollout': dt / reps * 1e3,
           'config': {'workload': 'E=%d, H=%d, obs=17, act=6, rollout_batch=%d per GPU, horizon=%d, %s terminations, '
                                  'penalty_coeff=%g, env pool %d rows' % (spec['E'], spec['H'], a2.batch, spec['h'],
                                                                           spec['domain'], spec['penalty'],
                                                                           spec['env_rows']),
                      'rollout_batch_per_gpu': a2.batch, 'horizon': spec['h']},
           'bnn_flop_per_row': fr,
           # rows per step shrink under terminations: transitions x flop/row bounds the ensemble rate from above
           'ensemble_algorithmic_tflops': v * fr / 1e12,
           'kernel_ms_avg': kms}
    if spec['domain'] == 'halfcheetah' or spec['h'] == 1:   # every ensemble launch runs all a2.batch rows
        out['roofline'] = leg_roofline(a2, kms)
    return out


def train_leg(args, env):
    """BNN.train minibatch steps (bnn.py:425-432) at the halfcheetah-mixed size: E=7, H=200, 101k env
    rows -> 100k train rows after the 1000-row holdout, batch 256 (mopo.py:529): 391 Adam steps per
    epoch.  Reports grad-steps/s over args.train_epochs timed epochs (+ the per-epoch holdout eval)."""
    import torch
    from mopo_amd.bnn import construct_model
    rs = np.random.RandomState(5)
    N = ENV_ROWS
    obs = env.cpu().numpy()
    act = rs.uniform(-1, 1, (N, A)).astype(np.float32)
    X = np.concatenate([obs, act], 1).astype(np.float32)
    Y = np.concatenate([rs.normal(size=(N, 1)), 0.1 * rs.normal(size=(N, O))], 1).astype(np.float32)
    m = construct_model(obs_dim=O, act_dim=A, hidden_dim=H, num_networks=E, num_elites=ELITES,
                        separate_mean_var=True, seed=1)
    x, y = torch.from_numpy(X).cuda(), torch.from_numpy(Y).cuda()
    np.random.seed(0)
    m.train(x, y, batch_size=256, max_epochs=1, holdout_ratio=0.2, permuted=True)   # warm-up + graph capture
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    m.train(x, y, batch_size=256, max_epochs=args.train_epochs, holdout_ratio=0.2, permuted=True)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    steps = m._train_grad_updates
    flop_step = 3 * 2 * E * 256 * ((O + A) * H + 3 * H * H + 2 * H * (O + 1))   # fwd + 2x bwd GEMMs
    return {'metric': 'BNN.train grad-steps/s (E=7, H=200, batch 256 per member)', 'value': steps / dt,
            'unit': 'grad-steps/s', 'ms_per_epoch': dt / args.train_epochs * 1e3, 'epochs_timed': args.train_epochs,
            'steps_per_epoch': steps // max(m._train_epochs, 1), 'train_rows': N - 1000,
            'tflops_achieved': steps * flop_step / dt / 1e12}


def cpu_baseline_train(args):
    """Oracle BNN training steps (numpy restatement of the TF graph, f32 arrays) on the host: median of 5
    runs of ``cpu_train_steps`` minibatch steps after a warm-up."""
    from oracle import bnn as obnn
    from oracle import bnn_train as ot
    rs = np.random.RandomState(0)
    p = obnn.init_params(E, O, A, hidden=H, seed=1)
    st = ot.TrainState(p, dtype=np.float32)
    X = rs.normal(size=(E, 256, O + A)).astype(np.float32)
    Y = rs.normal(size=(E, 256, O + 1)).astype(np.float32)
    n = args.cpu_train_steps

    def run():
        t0 = time.perf_counter()
        for _ in range(n):
            st.step(X, Y, np.float32)
        return n, time.perf_counter() - t0
    med, runs, units, secs = median_runs(run)
    return {'value': med, 'unit': 'grad-steps/s', 'cores': blas_threads(), 'kind': 'port', 'runs': runs, 'median': med,
            'sample': 'oracle numpy BNN train step (bnn.py:241-249 loss, hand backward, TF1 Adam), E=7, H=200, '
                      'batch 256: %d timed runs of %d steps (%.2f s) after 1 warm-up' % (CPU_RUNS, n, secs)}


SAC_DIAG = {}


def sac_roofline(rate):
    """one step is 0.59 GFLOP of GEMM work (forward + backward of the 8 MLP instances,
    oracle.sac.flops_per_step) and ~9.6 MB of parameter / Adam / target traffic; the floor is the larger
    of FLOP / f32 MFMA peak and bytes / HBM peak."""
    n, H_ = 256, HP
    pi_f, q_f = O * H_ + H_ * H_ + 2 * H_ * A, (O + A) * H_ + H_ * H_ + H_          # MACs per sample
    fwd = 2 * pi_f + 6 * q_f                       # pi(s), pi(s'), Q1/Q2 at (s, a), (s, pi(s)), target (s', pi')
    bwd = 2 * pi_f + 2 * (2 * q_f) + 2 * q_f      # pi params + input; Q1, Q2 params + input; Q*(s, pi) input
    fl = 2 * n * (fwd + bwd)
    n_par = (O * H_ + H_ + H_ * H_ + H_ + 2 * (H_ * A + A)) + 2 * ((O + A) * H_ + H_ + H_ * H_ + H_ + H_ + 1)
    by = n_par * 4 * 11     # params read + write, grads, Adam m / v read + write, target read + write
    floor_us = max(fl / (MFMA_F32_PEAK_TFLOPS * 1e12), by / 8e12) * 1e6
    us = 1e6 / rate
    return {'bound': 'latency (launch / dependency chain)', 'flop_per_step': fl, 'bytes_per_step': by,
            'floor_us': floor_us, 'achieved_us': us, 'frac': floor_us / us, 'traffic': sac_pmc_traffic(),
            'note': 'frac = max(FLOP / 157.3 TF f32 MFMA, bytes / 8 TB/s HBM) floor over the measured step time; '
                    'traffic = PMC HBM bytes per step (2 x FETCH_SIZE + WRITE_SIZE summed over the per-step SAC '
                    'launches) of the default workload, ' + os.path.relpath(PMC_SUMMARY, ROOT)}


def sac_pmc_traffic():
    """HBM bytes per SAC step from the committed PMC summary: the per-dispatch bytes of every per-step SAC
    launch (all ``mopo::sac_*`` kernels but the one-off batch gather and the logs read) summed, on the
    default C2 workload (product-default dtype) whose passes run 200 SAC steps (scripts/gpu_profile.sh)."""
    if not os.path.exists(PMC_SUMMARY):
        return None
    w = json.load(open(PMC_SUMMARY)).get('workloads', {}).get('C2 B=50000 h=5 dtype=%s' % DEFAULT_ENSEMBLE_DTYPE)
    if not w:
        return None
    ks = [v for k, v in w['kernels'].items()
          if k.startswith('mopo::sac_') and k not in ('mopo::sac_gather_kernel', 'mopo::sac_logs_kernel')]
    return sum(v['hbm_bytes'] for v in ks) if ks else None


def sac_leg(args, pool, env, dev, world):
    """SAC grad-steps/s: args.sac_steps x (_training_batch + _do_training + _update_target), graph replay."""
    import torch
    from mopo_amd.replay_pool import SimpleReplayPool
    from mopo_amd.sac import SAC
    env_pool = SimpleReplayPool(obs_dim=O, act_dim=A, max_size=ENV_ROWS)
    rs = np.random.RandomState(1)
    env_pool.add_samples({'observations': env[:ENV_ROWS], 'actions': rs.uniform(-1, 1, (ENV_ROWS, A)),
                          'next_observations': env[:ENV_ROWS] + 0.1 * torch.randn_like(env[:ENV_ROWS]),
                          'rewards': rs.normal(size=(ENV_ROWS, 1)), 'terminals': np.zeros((ENV_ROWS, 1), bool)})
    sac = SAC(O, A, HP, batch_size=256, real_ratio=0.05, target_entropy=-3)
    sac._do_training(0, env_pool, pool, n_steps=50, seed=5)
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    t0 = time.perf_counter()
    sac._do_training(50, env_pool, pool, n_steps=args.sac_steps, seed=5)
    t_enq = time.perf_counter() - t0
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        dt = float(t.item())
    lg = sac.logs()
    assert all(np.isfinite(v) for v in lg.values()), lg
    SAC_DIAG['enqueue_us_per_step'] = t_enq / args.sac_steps * 1e6
    return args.sac_steps / dt


def cpu_baseline_sac(args):
    """Oracle SAC steps (numpy restatement of mopo.py:204-466, 834-853) on the host, as BASELINE.md section 3
    times them: runs of ``cpu_sac_steps`` (1000) consecutive steps at batch 256 on one SAC state, the median
    of 5 timed runs after a warm-up run."""
    from oracle import sac as osac
    rs = np.random.RandomState(0)
    st = osac.SACState(osac.init_params(O, A, HP, seed=2, dtype=np.float32))
    for k in ('params', 'target'):
        setattr(st, k, [p.astype(np.float32) for p in getattr(st, k)])
    n = 256
    batch = {'observations': rs.normal(size=(n, O)).astype(np.float32), 'actions': rs.uniform(-1, 1, (n, A)).astype(np.float32),
             'next_observations': rs.normal(size=(n, O)).astype(np.float32), 'rewards': rs.normal(size=(n, 1)).astype(np.float32),
             'terminals': np.zeros((n, 1), bool)}
    per = max(args.cpu_sac_steps, 1)

    def run():
        t0 = time.perf_counter()
        for _ in range(per):
            osac.sac_step(st, batch, rs.normal(size=(n, A)).astype(np.float32), rs.normal(size=(n, A)).astype(np.float32))
        return per, time.perf_counter() - t0
    med, runs, units, secs = median_runs(run)
    return {'value': med, 'unit': 'grad-steps/s', 'cores': blas_threads(), 'kind': 'port', 'runs': runs, 'median': med,
            'steps_per_run': per,
            'sample': 'oracle numpy SAC step (fp32 arrays), batch 256: %d timed runs of %d consecutive steps (%.2f s) '
                      'after a warm-up run of %d' % (CPU_RUNS, per, secs, per)}


def main():
    args = parse()
    import torch
    rank, world, dev = dist_setup(args)
    model, pool, ro, pi, env, staging = build(args, dev, rank)
    for w in range(args.warmup):
        rollout_step(args, ro, pool, pi, env, staging, w, rank, world)
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    t0 = time.perf_counter()
    total = 0
    steps_t = []
    for s in range(args.steps):
        steps_t.append(rollout_step(args, ro, pool, pi, env, staging, args.warmup + s, rank, world))
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    dt = time.perf_counter() - t0
    total = int(sum(int(x.sum().item()) for x in steps_t))
    # per-kernel durations (HIP events on the rollout's stream around every launch) come from extra,
    # untimed rollouts: the event records themselves would add gaps to the timed region
    kernel_ms, _ = kernel_profile(args, ro, pool, pi, env, staging, args.warmup + args.steps, rank, world,
                                  args.prof_steps)
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        dt = float(t.item())
    sac_rate = sac_leg(args, pool, env, dev, world)
    extra = {}
    if rank == 0 and world == 1 and not args.no_c3 and args.config == 'C2':
        for key, name, dty in (('N2', 'N2', args.ensemble_dtype), ('N2_fp32', 'N2', 'fp32'), ('N2_f16x3', 'N2', 'f16x3'),
                               ('C3', 'C3', 'bf16'),
                               ('C4_per_gpu', 'C4', args.ensemble_dtype), ('C5_per_gpu', 'C5', 'fp32'),
                               ('C5_f16x3_per_gpu', 'C5', 'f16x3'), ('C5_bf16_per_gpu', 'C5', 'bf16')):
            extra[key] = config_leg(args, dev, name, dty)
    tr = train_leg(args, env) if (rank == 0 and world == 1 and args.train_epochs > 0 and args.config == 'C2') else None
    alts = {}
    if rank == 0 and world == 1 and not args.no_alt_dtypes and args.config == 'C2':
        for dt_alt in ('fp32', 'bf16x6', 'f16x3', 'bf16x3'):
            if dt_alt != args.ensemble_dtype:
                alts[dt_alt] = alt_headline_leg(args, dev, dt_alt)
    if rank != 0:
        if world > 1:
            torch.distributed.destroy_process_group()
        return
    value = total / dt
    spec = CONFIGS[args.config]
    out = {
        'metric': 'model-rollout transitions/s (halfcheetah-mixed)' if args.config == 'C2' else
                  'model-rollout transitions/s (%s: %s)' % (args.config, spec['name']),
        'value': value, 'unit': 'transitions/s', 'n_gpus': world, 'steps': args.steps, 'warmup': args.warmup,
        'ms_per_step': dt / args.steps * 1e3, 'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None,
        'dtype': dtype_desc(args.ensemble_dtype, args.actor_dtype), 'data': 'synthetic (random-init weights, N(0,1) env pool; D4RL/.mat unavailable offline)',
        'config': {'workload': '%s rollout: E=%d (5 elites), H=%d smv, obs=17, act=6, rollout_batch=%d per GPU, '
                               'horizon=%d, penalty_coeff=%g, learned-var penalty, env pool %d rows'
                               % (args.config, spec['E'], spec['H'], args.batch, args.horizon, spec['penalty'],
                                  spec['env_rows']),
                   'rollout_batch_per_gpu': args.batch, 'horizon': args.horizon, 'parallelism': 'dp%d' % world},
        'product_default_dtype': DEFAULT_ENSEMBLE_DTYPE,   # what MOPO.train / `mopo run_local` run
        'roofline': leg_roofline(args, kernel_ms),
        'kernel_ms_avg': kernel_ms,
        'sac': {'metric': 'SAC grad-steps/s (batch 256 = 12 env + 244 model rows, mopo.py:801-850)',
                'per_gpu': sac_rate, 'steps_timed': args.sac_steps,
                'us_per_step': 1e6 / sac_rate, **SAC_DIAG,
                'parallelism': 'replicated on every rank (the same updates on identical pools; SURVEY 8(e))',
                'roofline': sac_roofline(sac_rate)},
    }
    if extra:
        out['extra_configs'] = extra
    if alts:
        out['headline_other_dtypes'] = alts
    if tr is not None:
        out['model_train'] = tr
    if not args.no_cpu_baseline and world == 1:
        out['cpu_baseline'] = cpu_baseline(args)
        out['cpu_baseline_1core'] = cpu_baseline_1core(args)
        out['cpu_baseline_sac'] = cpu_baseline_sac(args)
        if args.train_epochs > 0:
            out['cpu_baseline_train'] = cpu_baseline_train(args)
    write_detail(args, out)
    print(json.dumps(compact_line(out)))
    if world > 1:
        torch.distributed.destroy_process_group()


LINE_LIMIT = 7000   # the driver keeps the last ~8 KB of stdout: the one bench line must fit in it whole


def _r(x, n=4):
    return None if x is None else float('%.*g' % (n, x))


def compact_line(out):
    """The one stdout line: the contract keys, the headline roofline, the CPU baseline, SAC, BNN.train and
    the credited-precision (fp32 / exact-operand) legs, each reduced to its figures.  Every leg in full
    (kernel tables, per-run CPU rates, sample descriptions) goes to the detail file (write_detail)."""
    keys = ('metric', 'value', 'unit', 'n_gpus', 'steps', 'warmup', 'ms_per_step', 'higher_is_better', 'scaling',
            'vs_baseline', 'dtype', 'data', 'config', 'product_default_dtype')
    line = {k: out[k] for k in keys if k in out}
    r = out['roofline']
    line['roofline'] = {'bound': r['bound'], 'achieved': _r(r['achieved']), 'peak': r['peak'], 'unit': r['unit'],
                        'frac': _r(r['frac']), 'traffic': r.get('traffic'),
                        'algorithmic_bytes': r.get('algorithmic_bytes_per_launch'),
                        'kernel': r['kernel'].split(' (')[0], 'avg_launch_ms': _r(r['avg_launch_ms'], 5),
                        'flop_per_launch': r.get('flop_per_launch')}
    line['kernel_ms_avg'] = {k: _r(v) for k, v in out['kernel_ms_avg'].items()}
    s = out['sac']
    line['sac'] = {'per_gpu': _r(s['per_gpu'], 5), 'us_per_step': _r(s['us_per_step'], 4),
                   'frac': _r(s['roofline']['frac']), 'floor_us': _r(s['roofline']['floor_us']),
                   'traffic': s['roofline'].get('traffic'), 'bytes_algorithmic': s['roofline']['bytes_per_step'],
                   'steps_timed': s['steps_timed']}
    if 'model_train' in out:
        t = out['model_train']
        line['model_train'] = {'value': _r(t['value'], 5), 'unit': t['unit'], 'ms_per_epoch': _r(t['ms_per_epoch']),
                               'tflops': _r(t['tflops_achieved'])}
    legs = {}
    for k, v in out.get('headline_other_dtypes', {}).items():
        legs['C2_' + k] = {'value': _r(v['value']), 'frac': _r(v['roofline']['frac']),
                           'ms': _r(v['roofline']['avg_launch_ms'])}
    for k, v in out.get('extra_configs', {}).items():
        rr = v.get('roofline')
        legs[k] = {'value': _r(v['value']), 'frac': _r(rr['frac']) if rr else None,
                   'ms': _r(rr['avg_launch_ms']) if rr else None}
    if legs:
        line['legs'] = legs
    if 'C2_fp32' in legs:
        line['fp32_leg'] = legs['C2_fp32']
    for k in ('cpu_baseline', 'cpu_baseline_1core', 'cpu_baseline_sac', 'cpu_baseline_train'):
        c = out.get(k)
        if not c:
            continue
        d = {'value': _r(c['value'], 5), 'unit': c['unit'], 'cores': c['cores'], 'kind': c['kind'],
             'median': _r(c['median'], 5), 'runs': [_r(x) for x in c['runs']]}
        if k == 'cpu_baseline':
            d['sample'] = c['sample']
            d['configs'] = {n: _r(v['value']) for n, v in c.get('configs', {}).items()}
        line[k] = d
    line['detail'] = 'every leg in full: gpurun_out/bench_detail.json (copied to profiles/r06_bench_full.json)'
    s = json.dumps(line)
    if len(s) > LINE_LIMIT:   # never let the headline fall out of the driver's tail
        for k in ('kernel_ms_avg', 'legs', 'cpu_baseline_1core'):
            line.pop(k, None)
    return line


def write_detail(args, out):
    """The full result (every leg, kernel tables, CPU-baseline runs) as one JSON file beside the bench line."""
    path = os.environ.get('MOPO_BENCH_DETAIL', os.path.join(ROOT, 'gpurun_out', 'bench_detail.json'))
    try:
        os.makedirs(os.path.dirname(path), exist_ok=True)
        with open(path, 'w') as f:
            json.dump(out, f, indent=1)
    except OSError as e:   # a read-only tree must not cost the bench line
        print('bench detail not written: %s' % e, file=sys.stderr)


def workload_key(args):
    return '%s B=%d h=%d dtype=%s' % (args.config, args.batch, args.horizon, args.ensemble_dtype)


def pmc_traffic(args):
    """HBM bytes per ensemble launch from the committed PMC summary (scripts/pmc.sh): the rollout-mode
    ensemble kernel (the most-dispatched ``mopo::bnn_fwd*``) of the passes collected on this exact
    workload; None when no pass ran on it."""
    if not os.path.exists(PMC_SUMMARY):
        return None
    w = json.load(open(PMC_SUMMARY)).get('workloads', {}).get(workload_key(args))
    if not w:
        return None
    cands = [(v.get('dispatches', 0), k) for k, v in w['kernels'].items() if k.startswith('mopo::bnn_fwd')]
    return w['kernels'][max(cands)[1]].get('hbm_bytes') if cands else None


from ctypes import c_double as C_double, c_int64 as C_int64  # noqa: E402

if __name__ == '__main__':
    main()
