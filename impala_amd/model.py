"""Actor-critic model whose parameters live in ONE flat fp32 buffer (state_dict order).

Mirrors ``models/distributed_models.py:12-32`` (``AtariPPOModel``: ``forward`` and the batched
``act``) over ``models/models.py:61-76`` / ``models/common.py:108-126`` (NatureCNN actor-critic).
Every parameter is a ``torch.nn.Parameter`` VIEW into ``self.flat`` (and every ``.grad`` a view
into ``self.flat_grad``) so that ``state_dict()`` / ``load_state_dict()`` / ``torch.save`` keep
the reference's key names, while the HIP library reads and updates the whole model through one
pointer.  The compute path is the HIP library only: ``forward`` on a non-GPU tensor raises.
"""
from __future__ import annotations

import os

import copy
import math
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch
import torch.nn as nn

OBS_SHAPE = (3, 64, 64)


def param_specs(num_actions: int = 15) -> List[Tuple[str, Tuple[int, ...]]]:
    """state_dict keys/shapes of the reference AtariPPOModel."""
    return [
        ("model.body.body.0.weight", (32, 3, 8, 8)),
        ("model.body.body.0.bias", (32,)),
        ("model.body.body.2.weight", (64, 32, 4, 4)),
        ("model.body.body.2.bias", (64,)),
        ("model.body.body.4.weight", (64, 64, 3, 3)),
        ("model.body.body.4.bias", (64,)),
        ("model.projection.0.weight", (1024,)),
        ("model.projection.0.bias", (1024,)),
        ("model.projection.1.weight", (256, 1024)),
        ("model.projection.1.bias", (256,)),
        ("model.actor.weight", (num_actions, 256)),
        ("model.actor.bias", (num_actions,)),
        ("model.critic.weight", (1, 256)),
        ("model.critic.bias", (1,)),
    ]


def param_count(num_actions: int = 15) -> int:
    return sum(int(np.prod(s)) for _, s in param_specs(num_actions))


class _Node(nn.Module):
    pass


def rebind_views(root: nn.Module, specs, flat: torch.Tensor, grad: Optional[torch.Tensor]) -> None:
    """Point every registered parameter of ``root`` (``specs`` order) back at its view of
    ``flat`` (and its ``.grad`` at the view of ``grad``).  Unpickling (``torch.load`` of a
    whole model) and ``copy.deepcopy`` rebuild each ``nn.Parameter`` on its own storage and
    drop ``.grad``; the HIP library reads and writes the model through the flat buffers only."""
    off = 0
    for name, shape in specs:
        cnt = int(np.prod(shape))
        param = root.get_parameter(name)
        param.data = flat[off:off + cnt].view(shape)
        param.grad = None if grad is None else grad[off:off + cnt].view(shape)
        off += cnt
    assert off == flat.numel()


# attributes holding native handles (ctypes pointers): never pickled, recreated lazily
ENGINE_ATTRS = ("_train_engine", "_infer_engine", "_engine")


def picklable_state(module: nn.Module) -> dict:
    state = dict(module.__dict__)
    for k in ENGINE_ATTRS:
        if k in state and not callable(state[k]):
            state[k] = None
    return state


class AtariPPOModel(nn.Module):
    """Drop-in for ``models.distributed_models.AtariPPOModel`` on an MI355X.

    ``forward(obs_u8[N,3,64,64]) -> (logits[N,A], v[N,1])`` through ``impala_forward``;
    ``act(obs, deterministic)`` as the reference's remote batched act (``:21-32``).
    """

    def __init__(self, observation_space: Tuple[int, ...] = OBS_SHAPE, action_dim: int = 15,
                 device="cuda", seed: Optional[int] = None, dtype: str = "fp32"):
        super().__init__()
        if tuple(observation_space) != OBS_SHAPE:
            # models/common.py:124-126 hard-codes output_dim 1024 => 64x64x3 only
            raise ValueError(f"AtariBody requires observations of shape {OBS_SHAPE}")
        if not 1 <= action_dim <= 15:
            raise ValueError("action_dim must be in [1, 15]")
        self.action_dim = action_dim
        self.compute_dtype = dtype
        device = torch.device(device)
        n = param_count(action_dim)
        self.flat = torch.zeros(n, dtype=torch.float32, device=device)
        self.flat_grad = torch.zeros(n, dtype=torch.float32, device=device)
        self._specs = param_specs(action_dim)
        self._views: Dict[str, Tuple[int, int, Tuple[int, ...]]] = {}
        self._version = 0          # bumped whenever self.flat changes
        self._train_engine = None  # Engine whose kernel-layout weights track every update
        self._infer_engine = None  # lazily created inference-only Engine
        # act() sampling stream; drawn outside torch's generator so seeded inits are unchanged
        self._act_seed = int.from_bytes(os.urandom(8), "little") >> 2
        off = 0
        for name, shape in self._specs:
            cnt = int(np.prod(shape))
            parts = name.split(".")
            mod = self
            for p in parts[:-1]:
                if not hasattr(mod, p) or not isinstance(getattr(mod, p), nn.Module):
                    mod.add_module(p, _Node())
                mod = getattr(mod, p)
            param = nn.Parameter(self.flat[off:off + cnt].view(shape))
            param.grad = self.flat_grad[off:off + cnt].view(shape)
            mod.register_parameter(parts[-1], param)
            self._views[name] = (off, cnt, shape)
            off += cnt
        assert off == n
        self.reset_parameters(seed)
        self.downstream = None

    # ---------------------------------------------------------------- parameters
    def reset_parameters(self, seed: Optional[int] = None) -> None:
        """Reference init, bit for bit: the layers are constructed in the reference's order on
        the CPU (each torch default init consumes the global RNG exactly as there) and
        ``layer_init_truncated`` is applied to the 3 convs and 3 Linears; LayerNorm stays
        (1, 0) (models/models.py:61-70, models/common.py:108-126,151-158).  ``seed`` seeds the
        global torch RNG first, as main.py:57-58 does before ``make_network``."""
        if seed is not None:
            torch.manual_seed(int(seed))
        std_div = np.asarray(.87962566103423978, dtype=np.float32)

        def trunc(layer, fan_in):
            with torch.no_grad():
                std = np.sqrt(1.0 / max(1, fan_in)) / std_div
                torch.nn.init.trunc_normal_(layer.weight, std=std)
                torch.nn.init.constant_(layer.bias, 0.)
            return layer

        layers = [trunc(nn.Conv2d(3, 32, 8, stride=4), 3 * 64),
                  trunc(nn.Conv2d(32, 64, 4, stride=2), 32 * 16),
                  trunc(nn.Conv2d(64, 64, 3, stride=1), 64 * 9)]
        ln = nn.LayerNorm(1024)
        layers += [ln, trunc(nn.Linear(1024, 256), 1024),
                   trunc(nn.Linear(256, self.action_dim), 256), trunc(nn.Linear(256, 1), 256)]
        flat = torch.cat([t.detach().reshape(-1) for l in layers for t in (l.weight, l.bias)])
        with torch.no_grad():
            self.flat.copy_(flat.to(self.flat.device))
        self.params_changed()

    def load_flat(self, flat) -> None:
        with torch.no_grad():
            self.flat.copy_(torch.as_tensor(np.asarray(flat, dtype=np.float32)).to(self.flat.device))
        self.params_changed()

    def params_changed(self) -> None:
        """Parameters were written from outside the HIP update: engines must re-derive their
        kernel-layout weights (lazily, before their next use)."""
        self._version = getattr(self, "_version", 0) + 1

    def load_state_dict(self, state_dict, strict: bool = True, assign: bool = False):
        res = super().load_state_dict(state_dict, strict=strict, assign=False)
        self.params_changed()
        return res

    # ---------------------------------------------------------------- pickling
    def __getstate__(self):
        """``torch.save(builder.learner_model)`` (reference main.py:117) works with engines
        attached: the engines hold native handles and are dropped (an unpickled model creates
        its inference engine lazily; a learner re-attaches its own)."""
        return picklable_state(self)

    def __setstate__(self, state):
        super().__setstate__(state)
        rebind_views(self, self._specs, self.flat, self.flat_grad)
        self.params_changed()

    # ---------------------------------------------------------------- compute
    def _engine(self):
        if self._train_engine is not None:
            return self._train_engine
        if self._infer_engine is None:
            from impala_amd.engine import Engine
            # the reference serves act() in batches of <= 128 (distributed_models.py:21)
            self._infer_engine = Engine(self, batch_size=2, rollout_length=64, inference_only=True)
        return self._infer_engine

    def forward(self, obs: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        """models/distributed_models.py:17-19 -> (logits [N,A], v [N,1])."""
        if obs.device.type != "cuda" or self.flat.device.type != "cuda":
            raise RuntimeError("AtariPPOModel.forward runs on the HIP path only (cuda device)")
        return self._engine().forward(obs)

    @torch.no_grad()
    def act(self, obs: torch.Tensor, deterministic_policy: torch.Tensor):
        """models/distributed_models.py:21-32: sample a ~ softmax(logits) (or argmax when
        deterministic); returns (action [N,1], logits [N,A], v [N,1]) on the CPU."""
        if self.flat.device.type != "cuda":
            raise RuntimeError("AtariPPOModel.act runs on the HIP path only (cuda device)")
        x = obs.to(self.flat.device)
        if x.dim() == 3:
            x = x.unsqueeze(0)
        # forward + argmax / softmax draw in one HIP call (impala_act); each call draws fresh
        self._act_calls = getattr(self, "_act_calls", 0) + 1
        action, logits, v = self._engine().act(x, deterministic_policy, seed=self._act_seed,
                                               counter=self._act_calls)
        # the three results to the host with one wait: asynchronous copies into page-locked
        # tensors (torch's caching host allocator), then a single stream synchronize -- instead
        # of three synchronous .cpu() round trips
        out = [torch.empty(t.shape, dtype=t.dtype, pin_memory=True) for t in (action, logits, v)]
        for h, t in zip(out, (action, logits, v)):
            h.copy_(t, non_blocking=True)
        torch.cuda.current_stream(self.flat.device).synchronize()
        return tuple(out)

    def push(self) -> None:
        """rlmeta DownstreamModel.push (utils.py:87-88): publish weights to the inference copy."""
        if self.downstream is not None:
            self.downstream.load_flat_from(self)

    def load_flat_from(self, other: "AtariPPOModel") -> None:
        with torch.no_grad():
            self.flat.copy_(other.flat.to(self.flat.device, non_blocking=True))
        self.params_changed()

    def clone_to(self, device) -> "AtariPPOModel":
        m = AtariPPOModel(OBS_SHAPE, self.action_dim, device=device, dtype=self.compute_dtype)
        m.load_flat_from(self)
        for p in m.parameters():
            p.requires_grad_(False)
        return m
