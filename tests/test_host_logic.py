"""Host-side logic on CPU: model parameter layout / init vs the reference fixtures, config
surface, replay semantics, collate, optimizer descriptor, actor trajectory format."""
import os

import numpy as np
import pytest
import torch

from impala_amd.config import load_config
from impala_amd.model import AtariPPOModel, param_count, param_specs
from impala_amd.replay import ReplayBuffer

G = os.path.join(os.path.dirname(__file__), "golden")


def test_param_specs_match_reference_state_dict():
    d = np.load(os.path.join(G, "model_forward.npz"), allow_pickle=False)
    assert [k for k, _ in param_specs(15)] == [str(k) for k in d["keys"]]
    assert param_count(15) == 344496


def test_model_views_and_reference_init_on_cpu():
    d = np.load(os.path.join(G, "model_forward.npz"), allow_pickle=False)
    m = AtariPPOModel((3, 64, 64), 15, device="cpu", seed=0)
    # bit-exact on the host that generated the fixture; torch's CPU erfinv goes through the host
    # libm's log, whose ifunc variant depends on the CPU, so other hosts differ by 1-2 ulp in
    # ~0.6 % of the weights (same bound as test_gpu_parity.py's init check)
    np.testing.assert_allclose(m.flat.numpy(), d["params"], rtol=1e-6, atol=1e-9)
    sd = m.state_dict()
    assert list(sd.keys()) == [str(k) for k in d["keys"]]
    # parameters and grads are views of the flat buffers
    w = m.model.body.body[0].weight if hasattr(m.model.body.body, "__getitem__") else \
        getattr(m.model.body.body, "0").weight
    assert w.data_ptr() == m.flat.data_ptr()
    assert w.grad.data_ptr() == m.flat_grad.data_ptr()
    # load_state_dict round trip writes through to the flat buffer
    sd2 = {k: torch.full_like(v, 0.5) for k, v in sd.items()}
    v0 = m._version
    m.load_state_dict(sd2)
    assert torch.all(m.flat == 0.5) and m._version > v0


def test_forward_refuses_cpu():
    m = AtariPPOModel((3, 64, 64), 15, device="cpu", seed=0)
    with pytest.raises(RuntimeError, match="HIP path only"):
        m(torch.zeros(1, 3, 64, 64, dtype=torch.uint8))


def test_model_rejects_non_64x64_observations():
    with pytest.raises(ValueError):
        AtariPPOModel((3, 84, 84), 15, device="cpu")


def test_config_surface_matches_reference_keys():
    c = load_config()
    assert c.agent.batch_size == 8 and c.agent.rollout_length == 20
    assert c.agent.learning_starts == 500  # deploy/local.yaml overlay
    assert c.agent.optimizer.lr == 1e-4 and c.agent.optimizer.eps == 1e-5
    assert c.agent.max_grad_norm == 40 and c.training.steps_per_epoch == 1000
    assert c.distributed.train_device == "cuda:0"
    c2 = load_config({"agent": {"batch_size": 64}, "learner": {"dtype": "fp32"}})
    assert c2.agent.batch_size == 64 and c2.learner.dtype == "fp32"


def _flatten(d, prefix=""):
    out = {}
    for k, v in d.items():
        if isinstance(v, dict):
            out.update(_flatten(v, f"{prefix}{k}."))
        else:
            out[f"{prefix}{k}"] = v
    return out


# keys this repo adds on top of the reference's files (everything else must match exactly)
_EXTRA_KEYS = {"config.yaml": ("learner.",), "agent/": ("name",)}


def test_conf_surface_matches_reference():
    """Every YAML file of the reference's conf/ exists here with the same keys and the same
    values (tests/golden/conf_keys.json, generated from the reference by make_conf_keys.py);
    additions are limited to the learner.* block and an agent `name`."""
    import json
    import yaml
    from impala_amd.config import CONF_DIR
    ref = json.load(open(os.path.join(G, "conf_keys.json")))
    for rel, want in ref.items():
        path = os.path.join(CONF_DIR, rel)
        assert os.path.exists(path), f"conf/{rel} missing"
        with open(path) as f:
            got = _flatten(yaml.safe_load(f) or {})
        extra = ()
        for pre, keys in _EXTRA_KEYS.items():
            if rel == pre or rel.startswith(pre):
                extra = keys
        added = [k for k in got if k not in want]
        assert all(any(k.startswith(e) for e in extra) for k in added), (rel, added)
        for k, v in want.items():
            assert k in got, f"conf/{rel}: key {k} missing"
            assert got[k] == v, f"conf/{rel}: {k} = {got[k]!r}, reference {v!r}"


def test_config_interpolations_and_groups():
    c = load_config()
    assert c.distributed.m_server_addr == "127.0.0.1:4411"  # conf/config.yaml:17
    assert c.distributed.r_server_addr == "127.0.0.1:4412"
    assert c.distributed.c_server_addr == "127.0.0.1:4413"
    assert c.hydra.run.dir == "." and c.hydra.output_subdir is None
    c2 = load_config({"distributed": {"server_addr": "10.0.0.2"}})
    assert c2.distributed.m_server_addr == "10.0.0.2:4411"
    assert load_config(agent="apex").agent.target_sync_period == 2500
    assert load_config(task="atari").task.env_id == "Breakout-v5"
    assert load_config(deploy="mila").distributed.host == "mila"
    assert load_config(deploy=None).agent.learning_starts == 100
    # the drop-in default computes in the reference's arithmetic
    assert load_config().learner.dtype == "fp32"


def _traj(T=20, A=15, fill=0):
    return [torch.full((T, 3, 64, 64), fill, dtype=torch.uint8),
            torch.zeros(T, 1, dtype=torch.int64), torch.zeros(T, 1), torch.zeros(T, 1),
            torch.zeros(T, A)]


def test_replay_circular_uniform_sampling():
    rb = ReplayBuffer(capacity=5, seed=1)
    for i in range(7):
        rb.append(_traj(fill=i))
    assert len(rb) == 5
    keys, batch, probs = rb.sample(4)
    assert len(set(keys.tolist())) == 4  # without replacement
    assert all(k >= 2 for k in keys)     # oldest two overwritten
    assert np.allclose(probs, 0.2)
    fills = sorted(int(b[0][0, 0, 0, 0]) for b in batch)
    assert all(2 <= f <= 6 for f in fills)


def test_replay_rows_carry_their_addresses():
    """ReplayBuffer.sample returns the reference's list of trajectories as a RowBatch that also
    carries each row's host address and layout key (what impala_stage_rows reads); a sample
    that includes a non-contiguous trajectory carries none."""
    from impala_amd.replay import RowBatch
    rb = ReplayBuffer(capacity=5, seed=1)
    for i in range(7):
        t = _traj(fill=i)
        t[2] = torch.full((20, 1), float(i))
        rb.append(t)
    keys, batch, probs = rb.sample(4)
    assert isinstance(batch, RowBatch) and len(batch) == 4 and np.allclose(probs, 0.2)
    assert all(k >= 2 for k in keys)
    assert batch.row_key == ((torch.uint8, torch.int64, torch.float32, torch.float32, torch.float32),
                             (20 * 3 * 64 * 64, 20 * 8, 20 * 4, 20 * 4, 20 * 15 * 4))
    for b, item in enumerate(batch):
        assert int(item[0][0, 0, 0, 0]) == int(keys[b]) == int(item[2][0, 0])
        for f in range(5):
            assert int(batch.row_ptrs[f][b]) == item[f].data_ptr()
    odd = _traj(fill=9)
    odd[4] = torch.zeros(15, 20).t()  # non-contiguous logits
    rb2 = ReplayBuffer(capacity=1, seed=0)
    rb2.append(odd)
    _, b2, _ = rb2.sample(1)
    assert b2.row_ptrs is None and b2.row_key is None


def test_agent_host_floats_one_copy_per_vector():
    """DistributedAgent turns a step's device metric scalars (views of one metrics vector, as
    ImpalaLearner returns them) into floats from one stacked copy, and plain values through
    float(v), with the values float(v) gives."""
    from impala_amd.agent import _host_floats
    vecs = [torch.arange(9, dtype=torch.float32) * (k + 1) for k in range(3)]
    pend = [dict(zip(("a", "b", "c"), v.unbind(0)), d=0.5, e=torch.tensor(2.0)) for v in vecs]
    got = _host_floats(pend)
    for k, g in enumerate(got):
        assert g == {"a": 0.0, "b": 1.0 * (k + 1), "c": 2.0 * (k + 1), "d": 0.5, "e": 2.0}


def test_replay_warm_up_times_out():
    rb = ReplayBuffer(capacity=4)
    rb.append(_traj())
    rb.warm_up(1)
    with pytest.raises(TimeoutError):
        rb.warm_up(3, timeout=0.05)


def test_collate_list_of_trajectories_on_cpu():
    from impala_amd.learner import _collate
    batch = [_traj(fill=i) for i in range(3)]
    obs, act, rew, disc, mu = _collate(batch, torch.device("cpu"))
    assert obs.shape == (3, 20, 3, 64, 64) and obs.dtype == torch.uint8
    assert act.shape == (3, 20) and act.dtype == torch.int64
    assert rew.shape == (3, 20) and disc.shape == (3, 20) and mu.shape == (3, 20, 15)
    assert int(obs[2, 0, 0, 0, 0]) == 2


def test_adam_descriptor_from_torch():
    from impala_amd.learner import ImpalaAdam
    p = torch.nn.Parameter(torch.zeros(3))
    a = ImpalaAdam.from_torch(torch.optim.Adam([p], lr=3e-4, eps=1e-5))
    assert a.lr == 3e-4 and a.eps == 1e-5 and a.betas == (0.9, 0.999)
    with pytest.raises(TypeError):
        ImpalaAdam.from_torch(torch.optim.SGD([p], lr=0.1))


def test_actor_make_replay_format():
    from impala_amd.builder import ImpalaActor

    class _RB:
        items = []

        def append(self, x):
            self.items.append(x)

    rb = _RB()
    actor = ImpalaActor(model=None, replay_buffer=rb, rollout_length=3)
    actor._last_transition = (torch.zeros(3, 64, 64, dtype=torch.uint8), 0.0, False)
    for t in range(3):
        nxt = (torch.full((3, 64, 64), t + 1, dtype=torch.uint8), 1.0, t == 1)
        actor.observe((torch.tensor([t]), {"logpi": torch.zeros(15)}), nxt)
    s, a, r, g, mu = rb.items[0]
    assert s.shape == (3, 3, 64, 64) and a.shape == (3, 1) and r.shape == (3, 1)
    assert mu.shape == (3, 15) and a.dtype == torch.int64
    np.testing.assert_allclose(g.squeeze(-1).numpy(), [0.99, 0.0, 0.99])  # (not done)*gamma


def test_shard_range():
    from impala_amd.distributed import shard_range
    assert shard_range(512, 8, 3) == (192, 256)
    with pytest.raises(ValueError):
        shard_range(10, 4, 0)


def test_ppo_collate_transitions_matches_torch_cat():
    """CircularBuffer(collate_fn=torch.cat) semantics (agents/ppo/builder.py:30-35)."""
    import torch
    from impala_amd.ppo import collate_transitions
    rng = np.random.default_rng(0)
    items = []
    for i in range(5):
        items.append([torch.from_numpy(rng.integers(0, 256, (1, 3, 64, 64), dtype=np.uint8)),
                      torch.tensor([i % 3]), torch.tensor([0.5 * i]),
                      torch.from_numpy(rng.standard_normal((1, 15)).astype(np.float32))])
    s, a, t, mu = collate_transitions(items, torch.device("cpu"))
    assert s.shape == (5, 3, 64, 64) and s.dtype == torch.uint8
    assert a.tolist() == [0, 1, 2, 0, 1] and a.dtype == torch.int64
    assert t.tolist() == [0.0, 0.5, 1.0, 1.5, 2.0]
    assert torch.equal(mu, torch.cat([x[3] for x in items]))
    # items without the leading dim collate the same way
    s2, a2, t2, mu2 = collate_transitions([[x[0][0], x[1][0], x[2][0], x[3][0]] for x in items],
                                          torch.device("cpu"))
    assert torch.equal(s2, s) and torch.equal(a2, a) and torch.equal(t2, t) and torch.equal(mu2, mu)


class _Ctl:
    """rlmeta controller stand-in (set_phase / reset_phase / count / stats / connect)."""

    def __init__(self):
        self.phases, self.n = [], 0

    def set_phase(self, phase):
        self.phases.append(phase)

    def reset_phase(self, phase, limit=None):
        self.limit = limit

    def count(self, phase):
        self.n += 2
        return self.n

    def stats(self, phase):
        from impala_amd.agent import StatsDict
        s = StatsDict()
        for x in (100, 200, 300):
            s.extend({"episode_length": x, "episode_return": x / 10})
        return s


class _Learner:
    samples_per_step = 160

    def __init__(self):
        self.steps = 0

    def prepare(self):
        pass

    def connect(self):
        pass

    def train_step(self):
        self.steps += 1
        return {"train/loss": torch.tensor(1.0 / self.steps)}


class _Writer:
    def __init__(self):
        self.logs = []

        class _Run:
            def log(run, d):
                self.logs.append(d)
        self.run = _Run()


def test_distributed_agent_train_returns_total_samples():
    """agents/distributed_agent.py:26-42: train returns total_samples = mean episode length x
    episode count from the controller's TRAIN stats and logs debug/total_samples,
    train_envs/* and debug/samples_per_second through writer.run.log."""
    from impala_amd.agent import DistributedAgent, Phase
    ctl, w = _Ctl(), _Writer()
    ag = DistributedAgent(ctl, _Learner(), w)
    total = ag.train(250)
    assert total == 200 * 3
    assert ctl.phases == [Phase.TRAIN]
    keys = [k for d in w.logs for k in d]
    assert keys.count("train/loss") == 3  # steps 0, 100, 200
    assert "debug/total_samples" in keys and "debug/samples_per_second" in keys
    assert "train_envs/episode_return" in keys
    assert ag.stats.dict()["train/loss"]["count"] == 250
    ev = ag.eval(num_episodes=6, keep_training_loops=False)
    assert ctl.phases[-1] == Phase.EVAL and ctl.limit == 6
    assert ev.dict()["episode_length"]["mean"] == 200
    # without a controller: the frames the learner consumed
    assert DistributedAgent(None, _Learner(), w).train(5) == 5 * 160


@pytest.mark.parametrize("A", [1, 2, 6, 9, 15])
def test_adam_block_partition_covers_every_parameter_once(A):
    """adam_kernel's block map (kernels.h: HID blocks of one FC weight row each, 4 parameters per
    thread, then one parameter per thread over [0, wfc) ++ [bfc, total)) restated on the host:
    every canonical parameter is updated by exactly one thread, the FC rows start float4-aligned,
    and the grid impala.hip launches (HID + cdiv(rest, 256)) is exactly enough."""
    specs = param_specs(A)
    sizes = [int(np.prod(s)) for _, s in specs]
    offs = np.concatenate([[0], np.cumsum(sizes)])
    seg = {n: (int(offs[i]), int(offs[i + 1])) for i, (n, _) in enumerate(specs)}
    total = int(offs[-1])
    wfc, bfc = seg["model.projection.1.weight"]
    HID, FLAT = 256, 1024
    assert bfc - wfc == HID * FLAT
    hits = np.zeros(total, np.int32)
    for o in range(HID):  # FC rows: thread t takes 4 t .. 4 t + 3
        c0 = wfc + o * FLAT
        assert c0 % 4 == 0
        for t in range(256):
            hits[c0 + 4 * t:c0 + 4 * t + 4] += 1
    rest = total - (bfc - wfc)
    for e in range(-(-rest // 256) * 256):  # the generic blocks
        i = e if e < wfc else e + (bfc - wfc)
        if i < total:
            hits[i] += 1
    assert (hits == 1).all(), np.nonzero(hits != 1)[0][:10]


def test_torchrun_launcher_binds_its_own_port(tmp_path):
    """tests/torchrun_util.py: the launcher's c10d store binds port 0 itself (--standalone on
    127.0.0.1), so no port number is chosen before the socket that uses it exists.  Two gloo
    ranks rendezvous through it and all-reduce."""
    import os
    import torchrun_util

    cmd = torchrun_util.torchrun_cmd("w.py", 2)
    assert "--standalone" in cmd and "--local-addr=127.0.0.1" in cmd
    assert not any(c.startswith("--master-port") for c in cmd)
    w = tmp_path / "w.py"
    w.write_text("import os, torch, torch.distributed as dist\n"
                 "dist.init_process_group('gloo')\n"
                 "t = torch.ones(1) * (dist.get_rank() + 1)\n"
                 "dist.all_reduce(t)\n"
                 "assert t.item() == 3.0 and os.environ['MASTER_ADDR'] == '127.0.0.1'\n"
                 "dist.destroy_process_group()\n")
    r = torchrun_util.torchrun(w, 2, dict(os.environ), str(tmp_path), timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
