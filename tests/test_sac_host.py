"""SAC boundary and host logic on CPU: include/sac_hip.h vs the
binding vs the library's exports, argument validation without a device, the parameter
layout / init vs the reference fixture, state_dict keys, the builder's config surface."""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest
import torch

from impala_amd import _lib

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "sac_hip.h")
G = os.path.join(REPO, "tests", "golden")


def _declared():
    src = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    return sorted(set(re.findall(r"\b(sac_\w+)\s*\(", src)))


def test_header_declares_what_the_binding_expects():
    assert _declared() == sorted(_lib.SAC_EXPORTS)


def test_library_exports_every_declared_symbol():
    lib = _lib.lib()
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r"\b(sac_\w+)\b", out))
    for name in _declared():
        assert name in exported, name
        assert hasattr(lib, name)


def test_struct_layouts_match_header():
    # the ctypes mirrors must have the header's field order and count
    src = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    body = re.search(r"typedef struct \{(.*?)\} sac_config;", src, flags=re.S).group(1)
    fields = re.findall(r"(\w+)(?:\s*,\s*(\w+))?(?:\s*,\s*(\w+))?;", body)
    names = [n for grp in fields for n in grp if n]
    assert names == [f for f, _ in _lib.SacConfig._fields_]
    body = re.search(r"typedef struct \{(.*?)\} sac_batch;", src, flags=re.S).group(1)
    assert re.findall(r"\*\s*(\w+);", body) == [f for f, _ in _lib.SacBatch._fields_]


def test_host_only_entry_points():
    lib = _lib.lib()
    assert lib.sac_actor_param_count(17, 6) == 73484
    assert lib.sac_critic_param_count(17, 6) == 144386
    cfg = _lib.SacConfig()
    assert lib.sac_config_default(C.byref(cfg)) == 0
    assert (cfg.obs_dim, cfg.act_dim, cfg.batch_size) == (17, 6, 256)
    assert abs(cfg.critic_lr - 3e-3) < 1e-9 and abs(cfg.actor_lr - 3e-4) < 1e-10
    assert abs(cfg.tau - 0.005) < 1e-9 and abs(cfg.max_grad_norm - 40) < 1e-6
    assert cfg.tune_alpha == 1 and abs(cfg.prio_exponent - 0.4) < 1e-7
    names = [lib.sac_phase_name(i).decode() for i in range(lib.sac_phase_count())]
    assert names[0] == "pack" and len(set(names)) == len(names)
    assert {"finalize", "critic_fwd_chain", "critic_loss_chain", "actor_chain"} <= set(names)
    assert lib.sac_phase_name(-1) is None


@pytest.mark.parametrize("field,value", [("obs_dim", 0), ("act_dim", 0), ("act_dim", 17),
                                         ("batch_size", 0), ("dtype", 5)])
def test_create_rejects_bad_config_without_touching_the_device(field, value):
    lib = _lib.lib()
    cfg = _lib.SacConfig()
    lib.sac_config_default(C.byref(cfg))
    setattr(cfg, field, value)
    h = C.c_void_p()
    assert lib.sac_create(C.byref(cfg), 0, C.byref(h)) == 1001
    assert not h.value
    assert lib.impala_last_error().decode().startswith("sac_create")


def test_entry_points_validate_before_launch():
    lib = _lib.lib()
    assert lib.sac_train_step(None, None, None) == 1001
    assert lib.sac_act(None, None, 1, None, 1.0, 1.0, 0.0, None, None) == 1001
    assert lib.sac_policy(None, None, 1, *([None] * 7)) == 1001
    assert lib.sac_q_forward(None, None, None, 1, 0, None, None, None) == 1001
    assert lib.sac_sample(0, 0, 0, 4, None, None, None, None, None, 0, None) == 1001
    assert lib.sac_bind_state(None, None, None) == 1001
    assert lib.sac_timer_start(None, 0, 1) == 1001


def test_modules_match_reference_init_and_keys_on_cpu():
    from impala_amd.sac import SoftActor, SoftCritic
    d = np.load(os.path.join(G, "sac_train_step.npz"), allow_pickle=False)
    torch.manual_seed(0)  # builder.py:60-66: critic first, then actor
    critic = SoftCritic((17,), (6,), device="cpu")
    actor = SoftActor((17,), (6,), device="cpu")
    np.testing.assert_array_equal(critic.flat.numpy(), d["critic0"])
    np.testing.assert_array_equal(critic.target_flat.numpy(), d["target0"])
    np.testing.assert_array_equal(actor.flat.numpy(), d["actor0"])
    assert float(critic.log_alpha) == float(d["log_alpha0"]) == 0.0
    keys = list(actor.state_dict().keys())
    assert keys[:2] == ["actor.body.body.0.weight", "actor.body.body.0.bias"]
    assert "actor.head.fc_logstd.bias" in keys and "actor.head.action_scale" in keys
    ck = list(critic.state_dict().keys())
    # nn.Module.state_dict: own parameters, own buffers, then children (as the reference's)
    assert ck[:3] == ["log_alpha", "target_entropy", "critic.q1.body.0.weight"]
    assert ck[-1] == "target_critic.q2.body.4.bias" and len(ck) == 2 + 24
    assert float(critic.target_entropy) == -6.0
    assert not any(p.requires_grad for p in critic.target_critic.parameters())
    # parameters are views of the flat buffers; grads of the grad buffers
    w = actor.actor.body.body[0].weight if hasattr(actor.actor.body.body, "__getitem__") else \
        getattr(actor.actor.body.body, "0").weight
    assert w.data_ptr() == actor.flat.data_ptr() and w.grad.data_ptr() == actor.flat_grad.data_ptr()
    assert critic.log_alpha.data_ptr() == critic.la_buf.data_ptr()
    # a deep copy (learning.py:134 target actor) owns its own flat buffer
    import copy
    t = copy.deepcopy(actor)
    assert t.flat.data_ptr() != actor.flat.data_ptr() and torch.equal(t.flat, actor.flat)
    v0 = actor._version
    actor.load_state_dict({k: torch.zeros_like(v) for k, v in actor.state_dict().items()})
    assert actor._version > v0 and float(actor.flat.abs().sum()) == 0.0


def test_compute_refuses_cpu():
    from impala_amd.sac import SoftActor
    actor = SoftActor((5,), (2,), device="cpu")
    with pytest.raises(RuntimeError):
        actor(torch.zeros(3, 5))
    with pytest.raises(RuntimeError):
        actor.act(torch.zeros(3, 5), 0.)


def test_builder_config_surface():
    from impala_amd.config import load_config
    cfg = load_config({"defaults": {}}, deploy=None)
    sac = load_config(agent="sac")
    a = sac.agent
    assert (a.batch_size, a.replay_buffer_size, a.push_period) == (256, 1000000, 5)
    assert abs(a.optimizer.critic_lr - 0.003) < 1e-12 and abs(a.optimizer.actor_lr - 0.0003) < 1e-12
    # conf/deploy/local.yaml overrides agent.learning_starts (5000 in sac.yaml) with 500
    assert a.tune_alpha is True and a.alpha == 1.0 and a.learning_starts == 500
    assert sac.task.env_id == "HalfCheetah-v4"
    assert cfg.agent.batch_size == 8  # default agent stays impala
