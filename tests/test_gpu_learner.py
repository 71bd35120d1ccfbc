"""GPU: the reference-shaped host API (ImpalaBuilder / ImpalaLearner / replay / model.act /
push / checkpoint) drives the HIP path and agrees with the oracle."""
import numpy as np
import pytest
import torch

from oracle import ref_cpu

pytestmark = pytest.mark.gpu


# impala_stage copy paths: the default (obs over 2 SDMA streams, the small fields in one pull
# launch), all SDMA copies, 3 obs streams, and the pull kernel for everything
H2D_MODES = {"default": {},
             "sdma_only": {"IMPALA_H2D_SMALL_PULL": "0"},
             "sdma_3streams": {"IMPALA_H2D_STREAMS": "3"},
             "pull8": {"IMPALA_H2D_KERNEL": "8"}}


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


class _FixedReplay:
    def __init__(self, batches):
        self.batches = list(batches)
        self.warm = None

    def warm_up(self, n):
        self.warm = n

    def sample(self, b):
        return None, self.batches.pop(0), None


def _cfg(**over):
    from impala_amd.config import load_config
    o = {"learner": {"dtype": "fp32"}}
    for k, v in over.items():
        o.setdefault(k, {}).update(v)
    return load_config(o)


# the drop-in path (ImpalaBuilder -> ImpalaLearner.train_step -> replay.sample -> host staging)
# against the float64 oracle, the yardstick test_gpu_parity_full.py uses.  Every step's metrics
# are checked against float64 run from the parameters the learner held before that step (the
# metrics are functions of the parameters and the batch): every key of every step within the
# north_star's 1e-5 relative, except train/pg, bounded NORMWISE (as test_gpu_parity_full.py
# bounds the V-trace outputs): |d| <= 1e-5 (|pg| + mean|log pi(a) adv|).  pg is a mean of
# mixed-sign terms of magnitude ~0.1-1 that cancels to -3e-3 at step 3 of this batch; there the
# fp32 path's 3.7e-7 absolute (1.2e-6 of the terms' mean magnitude, r06a) is 1.2e-4 of the
# cancelled value.  Over several steps the two trajectories part at rounding level (Adam turns a
# rounding-level difference in a near-zero gradient element into an O(lr) move), so the
# multi-step trajectory is bounded on the parameters, with test_gpu_parity_full.py's 3-step
# bound (max 5e-5, at most 100 parameters beyond 1e-6).
LEARNER_RTOL = 1e-5
KEYS = ("train/loss", "train/entropy", "train/td", "train/pg", "train/kl", "train/ratio",
        "train/grad_norm")


def test_builder_learner_step_matches_oracle():
    _dev()
    from impala_amd.builder import ImpalaBuilder
    B, T, steps = 4, 20, 4
    cfg = _cfg(agent={"batch_size": B})
    b = ImpalaBuilder(cfg)
    torch.manual_seed(0)
    model = b.make_network(None)
    flat0 = model.flat.cpu().numpy().copy()
    batch_np = ref_cpu.synthetic_batch(B, T, 15, seed=3)
    rb = _FixedReplay([ref_cpu.to_trajectories(*batch_np) for _ in range(steps)])
    learner = b.make_learner(model, rb)
    learner.prepare()
    assert rb.warm == cfg.agent.learning_starts
    traj = []
    p64, _, _ = ref_cpu.train_step_fp64(flat0, batch_np, 15, steps=steps, metrics_each=traj)
    worst, worst_traj, fails = {}, {}, []
    for step in range(steps):
        flat_k = model.flat.cpu().numpy().copy()
        cap = {}
        _, _, exp = ref_cpu.train_step_fp64(flat_k, batch_np, 15, steps=1, capture=cap)
        logp = torch.log_softmax(cap["logits"], -1).gather(
            -1, torch.from_numpy(batch_np[1]).unsqueeze(-1)).squeeze(-1)
        pg_scale = float((logp[:, :-1] * cap["adv"]).abs().mean())
        met = learner.train_step()
        for k in KEYS:
            got, want = float(met[k]), exp[k]
            scale = abs(want) + (pg_scale if k == "train/pg" else 0.0)
            rel = abs(got - want) / max(scale, 1e-30)
            worst[k] = max(worst.get(k, 0.0), rel)
            worst_traj[k] = max(worst_traj.get(k, 0.0),
                                abs(got - traj[step][k]) / max(abs(traj[step][k]), 1e-30))
            if rel > LEARNER_RTOL:
                fails.append((k, step, got, want, rel))
        for k in ("debug/replay_sample_per_second", "debug/gradient_per_second",
                  "debug/total_time", "debug/forward_dt", "debug/update_time"):
            assert k in met
    print("learner vs fp64 from the same parameters, worst rel over 4 steps (pg normwise): " +
          ", ".join(f"{k[6:]} {v:.2e}" for k, v in worst.items()))
    print("learner vs the fp64 4-step trajectory (for the record): " +
          ", ".join(f"{k[6:]} {v:.2e}" for k, v in worst_traj.items()))
    assert not fails, fails
    d = np.abs(model.flat.cpu().numpy() - p64)
    print(f"learner params after {steps} steps vs fp64: max |d| {d.max():.2e}, "
          f"n > 1e-6 {int(np.sum(d > 1e-6))}")
    assert d.max() <= 5e-5 and int(np.sum(d > 1e-6)) <= 100
    # push every model_push_period (4) steps: the actor copy now equals the learner weights
    torch.cuda.synchronize()
    np.testing.assert_array_equal(b.actor_model.flat.cpu().numpy(), model.flat.cpu().numpy())


def test_device_replay_gather_and_learn():
    dev = _dev()
    from impala_amd.replay import DeviceReplayBuffer
    T, A = 20, 15
    rb = DeviceReplayBuffer(capacity=16, rollout_length=T, num_actions=A, device=dev, seed=5)
    trajs = []
    for i in range(20):
        obs, act, rew, disc, mu = ref_cpu.synthetic_batch(1, T, A, seed=100 + i)
        item = [torch.from_numpy(obs[0]), torch.from_numpy(act[0]).unsqueeze(-1),
                torch.from_numpy(rew[0]).unsqueeze(-1), torch.from_numpy(disc[0]).unsqueeze(-1),
                torch.from_numpy(mu[0])]
        rb.append(item)
        trajs.append(item)
    rb.warm_up(10)
    keys, batch, probs = rb.sample(8)
    torch.cuda.synchronize()
    assert len(set(keys.tolist())) == 8 and all(k >= 4 for k in keys)
    for j, k in enumerate(keys.tolist()):
        src = trajs[k]
        np.testing.assert_array_equal(batch[0][j].cpu().numpy(), src[0].numpy())
        np.testing.assert_array_equal(batch[1][j].cpu().numpy(), src[1].squeeze(-1).numpy())
        np.testing.assert_array_equal(batch[2][j].cpu().numpy(), src[2].squeeze(-1).numpy())
        np.testing.assert_array_equal(batch[4][j].cpu().numpy(), src[4].numpy())
    from impala_amd.learner import ImpalaLearner
    from impala_amd.model import AtariPPOModel
    m = AtariPPOModel((3, 64, 64), A, device=dev, dtype="bf16", seed=0)
    ln = ImpalaLearner(m, rb, batch_size=8, rollout_length=T, learning_starts=10)
    ln.prepare()
    for _ in range(3):
        met = ln.train_step()
    assert np.isfinite(float(met["train/loss"]))


@pytest.mark.parametrize("h2d", sorted(H2D_MODES))
def test_host_staging_ring_matches_device_batches(h2d, monkeypatch):
    """impala_stage ring (2 slots, copies of step k+1 enqueued before step k; hipMemcpyAsync or
    the PCIe pull kernel) gives bitwise the same weights and metrics as the same batches handed
    over already in HBM."""
    dev = _dev()
    for k, v in H2D_MODES[h2d].items():
        monkeypatch.setenv(k, v)
    from impala_amd.engine import Engine
    from impala_amd.model import AtariPPOModel
    B, T, A, steps = 4, 20, 15, 5
    host = [[torch.from_numpy(x) for x in ref_cpu.synthetic_batch(B, T, A, seed=40 + s)]
            for s in range(steps)]

    def make():
        m = AtariPPOModel((3, 64, 64), A, device=dev, dtype="fp32", seed=0)
        e = Engine(m, batch_size=B, rollout_length=T, dtype="fp32")
        m._train_engine = e
        return m, e

    m1, e1 = make()
    for hb in host:
        e1.train_step(*[t.to(dev) for t in hb])
    m2, e2 = make()
    e2.stage_init(2)
    pinned = [[t.pin_memory() for t in hb] for hb in host]
    e2.stage(0, *pinned[0])
    for k in range(steps):
        s = k % 2
        if k + 1 < steps:
            e2.stage(1 - s, *pinned[k + 1])
        e2.train_step(e2.slot_batch(s))
        e2.slot_release(s)
    torch.cuda.synchronize()
    assert torch.equal(m1.flat, m2.flat)
    assert torch.equal(e1.metrics, e2.metrics)
    with pytest.raises(RuntimeError):
        e2.slot_batch(2)


def test_two_handles_share_the_copy_streams():
    """Two handles on one device share the staging copy streams (impala.hip acquire_h2d: one set
    per device and stream count, reference-counted).  Interleaved staging of different batches
    on both still gives each handle bitwise its device-batch result, and a handle keeps staging
    after the other is closed (the streams outlive the first handle's release)."""
    dev = _dev()
    from impala_amd.engine import Engine
    from impala_amd.model import AtariPPOModel
    B, T, A, steps = 4, 20, 15, 4
    batches = {w: [[torch.from_numpy(x) for x in ref_cpu.synthetic_batch(B, T, A, seed=70 + 10 * w + s)]
                   for s in range(2 * steps)] for w in (0, 1)}

    def make():
        m = AtariPPOModel((3, 64, 64), A, device=dev, dtype="fp32", seed=0)
        e = Engine(m, batch_size=B, rollout_length=T, dtype="fp32")
        m._train_engine = e
        return m, e

    refs = []
    for w in (0, 1):
        m, e = make()
        n = 2 * steps if w == 1 else steps
        for hb in batches[w][:n]:
            e.train_step(*[t.to(dev) for t in hb])
        torch.cuda.synchronize()
        refs.append((m.flat.clone(), e.metrics.clone()))
        e.close()
    pinned = {w: [[t.pin_memory() for t in hb] for hb in batches[w]] for w in (0, 1)}
    (m0, e0), (m1, e1) = make(), make()
    e0.stage_init(2)
    e1.stage_init(2)
    for k in range(steps):  # both rings in flight at once, on the shared streams
        s = k % 2
        e0.stage(s, *pinned[0][k])
        e1.stage(s, *pinned[1][k])
        e0.train_step(e0.slot_batch(s))
        e1.train_step(e1.slot_batch(s))
        e0.slot_release(s)
        e1.slot_release(s)
    torch.cuda.synchronize()
    assert torch.equal(m0.flat, refs[0][0]) and torch.equal(e0.metrics, refs[0][1])
    e0.close()
    for k in range(steps, 2 * steps):  # the other handle alone, after the first's release
        s = k % 2
        e1.stage(s, *pinned[1][k])
        e1.train_step(e1.slot_batch(s))
        e1.slot_release(s)
    torch.cuda.synchronize()
    assert torch.equal(m1.flat, refs[1][0]) and torch.equal(e1.metrics, refs[1][1])
    e1.close()


@pytest.mark.parametrize("A", [15, 6])
def test_native_act_argmax_flags_and_sampling_distribution(A):
    """impala_act (distributed_models.py:21-32): logits / values equal the forward, argmax where
    deterministic (per call or per frame), draws reproducible per (seed, counter), and the
    sampled frequencies follow softmax(logits) (chi-square)."""
    from scipy.stats import chisquare
    dev = _dev()
    from impala_amd.model import AtariPPOModel
    m = AtariPPOModel((3, 64, 64), A, device=dev, dtype="fp32", seed=1)
    e = m._engine()
    g = torch.Generator().manual_seed(0)
    obs = torch.randint(0, 256, (200, 3, 64, 64), dtype=torch.uint8, generator=g).to(dev)
    a, lg, v = e.act(obs, True)
    lg2, v2 = m(obs)
    assert torch.equal(lg, lg2) and torch.equal(v, v2)
    assert torch.equal(a.squeeze(1), lg.argmax(-1))
    flags = torch.zeros(200, dtype=torch.bool)
    flags[::2] = True
    a2, _, _ = e.act(obs, flags, seed=3, counter=1)
    assert torch.equal(a2[::2], a[::2])
    b1, _, _ = e.act(obs, False, seed=3, counter=5)
    b2, _, _ = e.act(obs, False, seed=3, counter=5)
    b3, _, _ = e.act(obs, False, seed=3, counter=6)
    assert torch.equal(b1, b2) and not torch.equal(b1, b3)
    assert int(b1.min()) >= 0 and int(b1.max()) < A
    # one frame's logits, many draws: frequencies vs softmax
    one = obs[:1].expand(128, 3, 64, 64).contiguous()
    counts = torch.zeros(A, dtype=torch.int64)
    for c in range(60):
        s, l1, _ = e.act(one, False, seed=11, counter=100 + c)
        counts += torch.bincount(s.squeeze(1).cpu(), minlength=A)
    p = torch.softmax(l1[0].double().cpu(), -1).numpy()
    n = int(counts.sum())
    assert chisquare(counts.numpy(), p * n).pvalue > 1e-4


def test_model_act_and_checkpoint_roundtrip(tmp_path):
    dev = _dev()
    from impala_amd.model import AtariPPOModel
    m = AtariPPOModel((3, 64, 64), 15, device=dev, dtype="fp32", seed=1)
    obs = torch.randint(0, 256, (130, 3, 64, 64), dtype=torch.uint8)
    a, lg, v = m.act(obs, torch.tensor([True]))
    assert a.shape == (130, 1) and lg.shape == (130, 15) and v.shape == (130, 1)
    assert torch.equal(a.squeeze(-1), lg.argmax(-1))
    a2, _, _ = m.act(obs, torch.tensor([False]))
    assert a2.shape == (130, 1) and int(a2.max()) < 15
    torch.save(m.state_dict(), tmp_path / "ck.pt")
    m2 = AtariPPOModel((3, 64, 64), 15, device=dev, dtype="fp32", seed=2)
    m2.load_state_dict(torch.load(tmp_path / "ck.pt", weights_only=True))
    lg1, v1 = m(obs.to(dev))
    lg2, v2 = m2(obs.to(dev))
    torch.testing.assert_close(lg1, lg2, rtol=0, atol=0)
    torch.testing.assert_close(v1, v2, rtol=0, atol=0)


def test_optimizer_state_resume_matches_uninterrupted():
    dev = _dev()
    from impala_amd.learner import ImpalaLearner
    from impala_amd.model import AtariPPOModel
    batches = [[torch.from_numpy(x).to(dev) for x in ref_cpu.synthetic_batch(2, 20, 15, seed=s)]
               for s in range(4)]

    def run(bs, model=None, state=None):
        m = model or AtariPPOModel((3, 64, 64), 15, device=dev, dtype="fp32", seed=0)
        ln = ImpalaLearner(m, _FixedReplay([tuple(b) for b in bs]), batch_size=2)
        if state is not None:
            ln.load_optimizer_state(state)
        for _ in range(len(bs)):
            ln.train_step()
        return m, ln

    m_full, _ = run(batches)
    m_a, ln_a = run(batches[:2])
    st = ln_a.optimizer_state()
    sd = {k: v.clone() for k, v in m_a.state_dict().items()}
    m_b = AtariPPOModel((3, 64, 64), 15, device=dev, dtype="fp32", seed=9)
    m_b.load_state_dict(sd)
    m_b, _ = run(batches[2:], m_b, st)
    torch.testing.assert_close(m_b.flat, m_full.flat, rtol=0, atol=0)


@pytest.mark.parametrize("h2d", sorted(H2D_MODES))
def test_learner_host_batches_distinct_per_step(h2d, monkeypatch):
    """ImpalaLearner.train_step on host (list-of-trajectories) batches reuses two page-locked
    staging buffers in place; with a DIFFERENT batch every step (hipMemcpyAsync or the PCIe
    pull kernel) the weights and metrics are bitwise those of the same batches handed over
    already in HBM -- a stale or torn read of a reused host buffer would show here."""
    dev = _dev()
    for k, v in H2D_MODES[h2d].items():
        monkeypatch.setenv(k, v)
    from impala_amd.engine import Engine
    from impala_amd.learner import ImpalaLearner
    from impala_amd.model import AtariPPOModel
    B, T, A, steps = 4, 20, 15, 6
    batches = [ref_cpu.synthetic_batch(B, T, A, seed=500 + s) for s in range(steps)]
    m1 = AtariPPOModel((3, 64, 64), A, device=dev, dtype="fp32", seed=0)
    ln = ImpalaLearner(m1, _FixedReplay([ref_cpu.to_trajectories(*b) for b in batches]),
                       batch_size=B, rollout_length=T, model_push_period=1000)
    mets = [ln.train_step() for _ in range(steps)]
    m2 = AtariPPOModel((3, 64, 64), A, device=dev, dtype="fp32", seed=0)
    e2 = Engine(m2, batch_size=B, rollout_length=T)
    m2._train_engine = e2
    for s, b in enumerate(batches):
        e2.train_step(*[torch.from_numpy(np.ascontiguousarray(x)).to(dev) for x in b])
        torch.cuda.synchronize()
        assert float(mets[s]["train/loss"]) == float(e2.metrics[0]), s
    torch.cuda.synchronize()
    assert torch.equal(m1.flat, m2.flat)


def test_device_replay_overwrite_waits_for_queued_gather():
    """An append into the slot a queued gather still reads must wait for that gather: fill a
    capacity-4 ring, sample all 4, immediately append into the oldest slot, then check the
    gathered batch holds the old trajectories (not the new one)."""
    dev = _dev()
    from impala_amd.replay import DeviceReplayBuffer
    T, A = 20, 15

    def item(i):
        obs, act, rew, disc, mu = ref_cpu.synthetic_batch(1, T, A, seed=900 + i)
        return [torch.from_numpy(obs[0]), torch.from_numpy(act[0]).unsqueeze(-1),
                torch.from_numpy(rew[0]).unsqueeze(-1), torch.from_numpy(disc[0]).unsqueeze(-1),
                torch.from_numpy(mu[0])]

    rb = DeviceReplayBuffer(capacity=4, rollout_length=T, num_actions=A, device=dev, seed=1)
    old = [item(i) for i in range(4)]
    for it in old:
        rb.append(it)
    torch.cuda.synchronize()
    # keep the learner stream busy so the gather is still queued when the append is issued
    busy = torch.randn(4096, 4096, device=dev)
    for _ in range(8):
        busy = busy @ busy
        busy = busy / busy.norm()
    keys, batch, _ = rb.sample(4)
    rb.append(item(99))  # overwrites slot 0 (key 0) on the replay's own stream
    torch.cuda.synchronize()
    for j, k in enumerate(keys.tolist()):
        np.testing.assert_array_equal(batch[0][j].cpu().numpy(), old[k][0].numpy())
        np.testing.assert_array_equal(batch[4][j].cpu().numpy(), old[k][4].numpy())


def test_device_replay_sample_never_waits_on_the_stream():
    """sample() holds the replay lock, so it must never wait on the device.  The
    sampled indices travel in the gather launch's arguments (impala_gather_rows_hidx): with
    the learner stream blocked behind queued work, ten samples in a row return while that work
    is still running, and every sample gathers the rows its keys name."""
    dev = _dev()
    from impala_amd.replay import DeviceReplayBuffer
    T, A = 4, 3
    rb = DeviceReplayBuffer(capacity=8, rollout_length=T, num_actions=A, device=dev, seed=2)
    for k in range(8):  # every field of trajectory k holds k
        rb.append([torch.full((T, 3, 64, 64), k, dtype=torch.uint8), torch.full((T, 1), k),
                   torch.full((T, 1), float(k)), torch.full((T, 1), float(k)),
                   torch.full((T, A), float(k))])
    torch.cuda.synchronize()
    busy = torch.randn(4096, 4096, device=dev)
    for _ in range(16):  # a few ms of queued work on the learner (current) stream
        busy = busy @ busy
        busy = busy / busy.norm()
    done = torch.cuda.Event()
    done.record()
    out = [rb.sample(4) for _ in range(10)]
    assert not done.query(), "sample() waited for the learner stream's queued work"
    torch.cuda.synchronize()
    for keys, batch, _ in out:
        for j, k in enumerate(keys.tolist()):
            assert int(batch[0][j].float().mean().item()) == k
            assert float(batch[4][j].mean().item()) == float(k)


def test_gather_rows_host_and_device_indices_agree():
    """impala_gather_rows (device indices) and impala_gather_rows_hidx (indices in the launch
    arguments, 256 rows per launch) copy the same rows: 300 rows of fields with row sizes
    below, at and above the 16 KB piece."""
    dev = _dev()
    from impala_amd.engine import gather_rollouts
    g = torch.Generator(device=dev).manual_seed(1)
    fields = [torch.randint(0, 255, (50, 3 * 16384 + 64), dtype=torch.uint8, device=dev, generator=g),
              torch.randn(50, 20, device=dev, generator=g),
              torch.randint(0, 1 << 30, (50, 16384 // 8), dtype=torch.int64, device=dev, generator=g)]
    idx = np.random.default_rng(0).integers(0, 50, size=300)
    a = gather_rollouts(fields, idx)
    b = gather_rollouts(fields, torch.from_numpy(idx).to(dev))
    ti = torch.from_numpy(idx).to(dev)
    for f, x, y in zip(fields, a, b):
        assert torch.equal(x, f[ti]) and torch.equal(y, f[ti])


def test_device_replay_append_during_sample_threaded():
    """appends racing sample() from another thread never tear a trajectory.  Every
    field of trajectory k encodes k, a capacity-8 ring is overwritten continuously by a writer
    thread while the main thread samples; each sampled row must be one whole trajectory and the
    one its returned key names."""
    import threading
    dev = _dev()
    from impala_amd.replay import DeviceReplayBuffer
    T, A, C = 20, 15, 8

    def item(k):
        return [torch.full((T, 3, 64, 64), k % 251, dtype=torch.uint8),
                torch.full((T, 1), k % A, dtype=torch.int64),
                torch.full((T, 1), float(k)), torch.full((T, 1), 0.5 * k),
                torch.full((T, A), float(-k))]

    rb = DeviceReplayBuffer(capacity=C, rollout_length=T, num_actions=A, device=dev, seed=3,
                            staging_slots=4)
    for k in range(C):
        rb.append(item(k))
    stop = threading.Event()
    errors = []

    def writer():
        k = C
        try:
            while not stop.is_set() and k < 5000:
                rb.append(item(k))
                k += 1
        except Exception as e:  # surfaced below
            errors.append(e)

    th = threading.Thread(target=writer)
    th.start()
    try:
        for _ in range(150):
            keys, (obs, act, rew, disc, mu), _ = rb.sample(C)
            torch.cuda.synchronize()
            r = rew.cpu().numpy()
            for j, k in enumerate(keys.tolist()):
                assert np.all(r[j] == float(k)), (j, k, r[j][:3])
                assert np.all(obs[j].cpu().numpy() == k % 251)
                assert np.all(act[j].cpu().numpy() == k % A)
                assert np.all(disc[j].cpu().numpy() == 0.5 * k)
                assert np.all(mu[j].cpu().numpy() == -float(k))
    finally:
        stop.set()
        th.join()
    assert not errors, errors


def test_device_replay_rows_read_during_appends_threaded():
    """The in-place read (sample_rows, then read_rows -- the path impala_train_step_rows takes)
    against a writer thread overwriting a capacity-8 ring: every row read is one whole
    trajectory (all five fields encode the same k), from the drawn slot, and the drawn one or a
    later one (a slot overwritten between the draw and the read is read with its new
    trajectory)."""
    import threading
    dev = _dev()
    from impala_amd.replay import DeviceReplayBuffer
    T, A, C = 20, 15, 8

    def item(k):
        return [torch.full((T, 3, 64, 64), k % 251, dtype=torch.uint8),
                torch.full((T, 1), k % A, dtype=torch.int64),
                torch.full((T, 1), float(k)), torch.full((T, 1), 0.5 * k),
                torch.full((T, A), float(-k))]

    rb = DeviceReplayBuffer(capacity=C, rollout_length=T, num_actions=A, device=dev, seed=4,
                            staging_slots=4)
    for k in range(C):
        rb.append(item(k))
    stop = threading.Event()
    errors = []

    def writer():
        k = C
        try:
            while not stop.is_set() and k < 5000:
                rb.append(item(k))
                k += 1
        except Exception as e:  # surfaced below
            errors.append(e)

    th = threading.Thread(target=writer)
    th.start()
    try:
        for _ in range(150):
            keys, rs, _ = rb.sample_rows(C)
            obs, act, rew, disc, mu = rs.gather()
            torch.cuda.synchronize()
            r = rew.cpu().numpy()
            for j, (slot, key) in enumerate(zip(rs.idx.tolist(), keys.tolist())):
                k = int(r[j][0])
                assert np.all(r[j] == float(k)), (j, r[j][:3])
                assert k % C == slot and k >= key, (j, slot, key, k)
                assert np.all(obs[j].cpu().numpy() == k % 251)
                assert np.all(act[j].cpu().numpy() == k % A)
                assert np.all(disc[j].cpu().numpy() == 0.5 * k)
                assert np.all(mu[j].cpu().numpy() == -float(k))
    finally:
        stop.set()
        th.join()
    assert not errors, errors


def test_whole_model_checkpoint_after_learner_step(tmp_path):
    """reference main.py:117 torch.save(builder.learner_model, ...) with the learner's engine
    (a native handle) attached: the model pickles, reloads with its parameters and gradients
    still views of the flat buffers, and serves forward through a fresh engine."""
    dev = _dev()
    from impala_amd.learner import ImpalaLearner
    from impala_amd.model import AtariPPOModel
    B, T = 2, 20
    batch = ref_cpu.synthetic_batch(B, T, 15, seed=77)
    m = AtariPPOModel((3, 64, 64), 15, device=dev, dtype="fp32", seed=0)
    ln = ImpalaLearner(m, _FixedReplay([ref_cpu.to_trajectories(*batch)]), batch_size=B,
                       rollout_length=T)
    ln.train_step()
    obs = torch.from_numpy(batch[0][0]).to(dev)
    lg0, v0 = m(obs)
    torch.save(m, tmp_path / "model.pt")
    m2 = torch.load(tmp_path / "model.pt", weights_only=False)  # our own file
    assert m2._train_engine is None and m2._infer_engine is None
    assert torch.equal(m2.flat, m.flat)
    w = m2.get_parameter("model.projection.1.weight")
    off = m2._views["model.projection.1.weight"][0]
    assert w.data_ptr() == m2.flat[off:].data_ptr()
    assert w.grad.data_ptr() == m2.flat_grad[off:].data_ptr()
    lg1, v1 = m2(obs)
    assert torch.equal(lg0, lg1) and torch.equal(v0, v1)


@pytest.mark.parametrize("mode", ["collate", "rows"])
def test_replay_rows_staged_match_device_batches(mode, monkeypatch):
    """ImpalaLearner over the host ReplayBuffer: each step's B trajectories are staged by
    impala_stage_rows from their own host rows -- collated by the library's thread pool into the
    slot's page-locked block (default), or one SDMA copy per row (IMPALA_STAGE_ROWS=rows).  An
    actor-side append replaces the oldest trajectory before every step while the learner
    prefetches ahead.  Weights and metrics must be bitwise those of the same trajectories (as
    sampled) handed over already collated in HBM."""
    dev = _dev()
    monkeypatch.setenv("IMPALA_STAGE_ROWS", mode)
    from impala_amd.engine import Engine
    from impala_amd.learner import ImpalaLearner
    from impala_amd.model import AtariPPOModel
    from impala_amd.replay import ReplayBuffer
    B, T, A, C, steps = 4, 20, 15, 6, 8
    trajs = [ref_cpu.to_trajectories(*ref_cpu.synthetic_batch(1, T, A, seed=700 + i))[0]
             for i in range(C + steps)]
    rb = ReplayBuffer(capacity=C, seed=4)
    for i in range(C):
        rb.append(trajs[i])
    seen = []
    sample = rb.sample

    def recording_sample(n):
        keys, batch, probs = sample(n)
        assert batch.row_ptrs is not None
        seen.append(keys.copy())
        return keys, batch, probs

    rb.sample = recording_sample
    m1 = AtariPPOModel((3, 64, 64), A, device=dev, dtype="fp32", seed=0)
    ln = ImpalaLearner(m1, rb, batch_size=B, rollout_length=T, model_push_period=1000)
    mets = []
    for s in range(steps):
        mets.append(ln.train_step())
        rb.append(trajs[C + s])  # replaces the oldest trajectory (the learner sampled ahead)
    m2 = AtariPPOModel((3, 64, 64), A, device=dev, dtype="fp32", seed=0)
    e2 = Engine(m2, batch_size=B, rollout_length=T)
    m2._train_engine = e2
    for s, (keys, met) in enumerate(zip(seen, mets)):  # (the last sample is the prefetch)
        items = [trajs[int(k)] for k in keys]
        b = [torch.stack([it[j] for it in items]).to(dev) for j in range(5)]
        b = [x.squeeze(-1) if j in (1, 2, 3) else x for j, x in enumerate(b)]
        e2.train_step(*[x.contiguous() for x in b])
        torch.cuda.synchronize()
        assert float(met["train/loss"]) == float(e2.metrics[0]), s
    torch.cuda.synchronize()
    assert torch.equal(m1.flat, m2.flat)


def test_agent_train_over_learner_floats_match_device_metrics():
    """DistributedAgent.train over ImpalaLearner (distributed_agent.py:26-41): the stats it
    folds in, read through one copy per step (sync_every 1) or per 3 steps, equal float(v) of
    the learner's own device metrics."""
    dev = _dev()
    from impala_amd.agent import DistributedAgent
    from impala_amd.learner import ImpalaLearner
    from impala_amd.model import AtariPPOModel
    B, T = 2, 20
    batches = [tuple(torch.from_numpy(x).to(dev) for x in ref_cpu.synthetic_batch(B, T, 15, seed=s))
               for s in range(5)]
    for sync in (1, 3):
        m = AtariPPOModel((3, 64, 64), 15, device=dev, dtype="fp32", seed=0)
        ln = ImpalaLearner(m, _FixedReplay(list(batches)), batch_size=B)
        got = []
        step = ln.train_step

        def recording():
            met = step()
            got.append({k: float(v) for k, v in met.items() if k.startswith("train/")})
            return met

        ln.train_step = recording
        ag = DistributedAgent(None, ln, sync_every=sync)
        ag.train(5)
        st = ag.stats.dict()
        for k in got[0]:
            assert st[k]["count"] == 5
            assert abs(st[k]["mean"] - sum(g[k] for g in got) / 5) <= 1e-6 * (1 + abs(st[k]["mean"]))
            assert st[k]["min"] == min(g[k] for g in got) and st[k]["max"] == max(g[k] for g in got)


def test_host_metrics_rows_match_device_vectors(monkeypatch):
    """impala_set_metrics_host: the row of the page-locked ring the step's last kernel writes
    is bitwise the step's device metrics vector; a row handed to a later step reads as None
    (the ring of 4 here), and DistributedAgent then falls back to the device copy -- its stats
    over a mix of both equal float(v) of every step."""
    dev = _dev()
    import impala_amd.learner as lmod
    from impala_amd import _lib
    from impala_amd.agent import DistributedAgent
    from impala_amd.model import AtariPPOModel
    monkeypatch.setattr(lmod, "HOST_METRICS_RING", 4)
    B, T, n = 2, 20, 12
    batches = [tuple(torch.from_numpy(x).to(dev) for x in ref_cpu.synthetic_batch(B, T, 15, seed=s))
               for s in range(n)]
    m = AtariPPOModel((3, 64, 64), 15, device=dev, dtype="fp32", seed=0)
    ln = lmod.ImpalaLearner(m, _FixedReplay(list(batches)), batch_size=B)
    mets = [ln.train_step() for _ in range(n)]
    torch.cuda.synchronize()
    for i, met in enumerate(mets):
        assert met.host is not None and met.host.index == i
        vals = met.host.values()
        if vals is not None:
            assert met.host.row.view(np.uint32)[15] == 1  # the ready word
        dev_vals = met["train/loss"]._base.cpu().tolist()
        if i >= n - 3:
            assert vals == dev_vals[:_lib.NUM_METRICS], i
            assert vals[7] == float(i + 1)  # the Adam step count
        else:
            assert vals is None, i
    for sync in (1, 6):
        m = AtariPPOModel((3, 64, 64), 15, device=dev, dtype="fp32", seed=0)
        ln = lmod.ImpalaLearner(m, _FixedReplay(list(batches)), batch_size=B)
        got = []
        step = ln.train_step

        def keep():
            met = step()
            got.append(met)
            return met

        ln.train_step = keep
        agent = DistributedAgent(None, ln, sync_every=sync)
        agent.train(n)
        torch.cuda.synchronize()
        floats = [{k: float(v) for k, v in g.items() if k.startswith("train/")} for g in got]
        stats = agent.stats.dict()
        for k in floats[0]:
            assert stats[k]["count"] == n
            assert stats[k]["min"] == min(f[k] for f in floats), (sync, k)
            assert stats[k]["max"] == max(f[k] for f in floats), (sync, k)
            mean = sum(f[k] for f in floats) / n
            assert abs(stats[k]["mean"] - mean) <= 1e-6 * (1 + abs(mean)), (sync, k)


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_train_step_rows_matches_the_gathered_batch(dtype):
    """impala_train_step_rows: the step on ring slots read in place (duplicates included) is
    bitwise the step on the same rows gathered into a batch; an out-of-range slot is refused
    before anything is enqueued."""
    dev = _dev()
    from impala_amd import _lib
    from impala_amd.engine import Engine, gather_rollouts
    from impala_amd.model import AtariPPOModel
    from impala_amd.replay import DeviceReplayBuffer
    B, T, A, C = 8, 20, 15, 24
    rb = DeviceReplayBuffer(C, T, A, device=dev, seed=3)
    for i in range(C):
        rb.append(ref_cpu.to_trajectories(*ref_cpu.synthetic_batch(1, T, A, seed=300 + i))[0])
    torch.cuda.synchronize()
    rng = np.random.default_rng(7)
    idxs = [rng.integers(0, C, size=B) for _ in range(4)]
    idxs[1][3] = idxs[1][5]  # a slot twice in one batch

    def make():
        m = AtariPPOModel((3, 64, 64), A, device=dev, dtype=dtype, seed=0)
        e = Engine(m, batch_size=B, rollout_length=T, dtype=dtype)
        m._train_engine = e
        return m, e

    m1, e1 = make()
    m2, e2 = make()
    for idx in idxs:
        e1.train_step(*gather_rollouts(rb.fields, idx))
        e2.train_step_rows(rb.fields, idx)
    torch.cuda.synchronize()
    assert torch.equal(m1.flat, m2.flat)
    assert torch.equal(e1.metrics, e2.metrics)
    bad = idxs[0].copy()
    bad[2] = C
    with pytest.raises(RuntimeError, match="out of range"):
        e2.train_step_rows(rb.fields, bad)
    assert torch.equal(m1.flat, m2.flat)


def test_learner_reads_device_replay_rows_in_place(monkeypatch):
    """ImpalaLearner over a DeviceReplayBuffer reads the sampled slots in place (no gather):
    bitwise the learner that gathers them (IMPALA_REPLAY_ROWS=0), with appends between the
    steps (prefetch 0: sampled and read at the step) and without (prefetch 2); and a handle on
    non-default kernels (IMPALA_FWD_FUSED=0) falls back to gathers with the same result."""
    dev = _dev()
    from impala_amd.learner import ImpalaLearner
    from impala_amd.model import AtariPPOModel
    from impala_amd.replay import DeviceReplayBuffer
    B, T, A, C, steps = 4, 20, 15, 12, 5
    trajs = [ref_cpu.to_trajectories(*ref_cpu.synthetic_batch(1, T, A, seed=900 + i))[0]
             for i in range(C + steps)]

    def run(rows, prefetch, appends, env=None):
        monkeypatch.setenv("IMPALA_REPLAY_ROWS", "1" if rows else "0")
        if env:
            monkeypatch.setenv(*env)
        rb = DeviceReplayBuffer(C, T, A, device=dev, seed=9)
        for t in trajs[:C]:
            rb.append(t)
        m = AtariPPOModel((3, 64, 64), A, device=dev, dtype="fp32", seed=0)
        ln = ImpalaLearner(m, rb, batch_size=B, rollout_length=T, prefetch=prefetch)
        losses = []
        for k in range(steps):
            losses.append(ln.train_step()["train/loss"])
            if appends:
                rb.append(trajs[C + k])
        torch.cuda.synchronize()
        if env:
            monkeypatch.delenv(env[0])
        return m.flat.clone(), [float(x) for x in losses], ln._rows_ok

    for prefetch, appends in ((0, True), (2, False)):
        p0, l0, ok0 = run(False, prefetch, appends)
        p1, l1, ok1 = run(True, prefetch, appends)
        assert not ok0 and ok1
        assert l0 == l1, (prefetch, appends)
        assert torch.equal(p0, p1), (prefetch, appends)
    p2, l2, ok2 = run(True, 2, False, env=("IMPALA_FWD_FUSED", "0"))
    p3, l3, _ = run(False, 2, False, env=("IMPALA_FWD_FUSED", "0"))
    assert ok2 is False  # fell back
    assert l2 == l3 and torch.equal(p2, p3)


@pytest.mark.parametrize("kind", ["device", "host_list"])
def test_learner_prefetch_matches_sampling_inside_the_step(kind):
    """ImpalaLearner(prefetch=1 or 2) samples and stages the next steps' batches right after a
    step is enqueued; with no appends in between it samples the same sequence as prefetch=0 (the
    reference's order, learning.py:121), so weights and metrics are bitwise equal, for each
    replay the learner can be given.  No step is waited for inside the loop, so a batch buffer
    reused while a queued step still reads it would show."""
    dev = _dev()
    from impala_amd.learner import ImpalaLearner
    from impala_amd.model import AtariPPOModel
    from impala_amd.replay import DeviceReplayBuffer, ReplayBuffer
    B, T, A, C, steps = 4, 20, 15, 12, 5
    trajs = [ref_cpu.to_trajectories(*ref_cpu.synthetic_batch(1, T, A, seed=800 + i))[0]
             for i in range(C)]

    def run(prefetch):
        rb = {"device": lambda: DeviceReplayBuffer(C, T, A, device=dev, seed=9),
              "host_list": lambda: ReplayBuffer(C, seed=9)}[kind]()
        for t in trajs:
            rb.append(t)
        m = AtariPPOModel((3, 64, 64), A, device=dev, dtype="fp32", seed=0)
        ln = ImpalaLearner(m, rb, batch_size=B, rollout_length=T, prefetch=prefetch)
        losses = [ln.train_step()["train/loss"] for _ in range(steps)]
        torch.cuda.synchronize()
        return m.flat.clone(), [float(x) for x in losses]

    p0, l0 = run(0)
    for depth in (1, 2):
        p1, l1 = run(depth)
        assert l0 == l1, depth
        assert torch.equal(p0, p1), depth
