"""Config tree with the reference's Hydra keys (conf/config.yaml:1-46, conf/agent/impala.yaml,
conf/deploy/local.yaml, conf/task/procgen.yaml), loaded with yaml.safe_load (Hydra is not a
dependency).  Attribute access like OmegaConf: ``cfg.agent.batch_size``."""
from __future__ import annotations

import copy
import os
from typing import Any, Dict, Optional

import yaml

CONF_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "conf")


class Cfg(dict):
    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def __setattr__(self, k, v):
        self[k] = v

    @staticmethod
    def wrap(x):
        if isinstance(x, dict):
            return Cfg({k: Cfg.wrap(v) for k, v in x.items()})
        if isinstance(x, list):
            return [Cfg.wrap(v) for v in x]
        return x


def _merge(a: Dict[str, Any], b: Dict[str, Any]) -> Dict[str, Any]:
    out = copy.deepcopy(a)
    for k, v in (b or {}).items():
        if isinstance(v, dict) and isinstance(out.get(k), dict):
            out[k] = _merge(out[k], v)
        else:
            out[k] = copy.deepcopy(v)
    return out


def _load(path):
    with open(path) as f:
        return yaml.safe_load(f) or {}


def _num(x):
    if isinstance(x, str):
        try:
            return float(x) if any(c in x for c in ".eE") else int(x)
        except ValueError:
            return x
    if isinstance(x, dict):
        return {k: _num(v) for k, v in x.items()}
    return x


def load_config(overrides: Optional[Dict[str, Any]] = None, deploy: Optional[str] = None,
                agent: Optional[str] = None, task: Optional[str] = None) -> Cfg:
    """Compose config.yaml + agent + task + deploy overlay (+ overrides), as main.py:39-53.
    ``agent`` / ``task`` select the group files as Hydra's ``agent=sac task=mujoco`` would
    (agent=sac alone implies task=mujoco, the reference's SAC task)."""
    base = _load(os.path.join(CONF_DIR, "config.yaml"))
    defaults = base.pop("defaults", {})
    cfg = dict(base)
    agent = agent or defaults.get("agent", "impala")
    task = task or ("mujoco" if agent == "sac" else defaults.get("task", "procgen"))
    cfg["agent"] = _load(os.path.join(CONF_DIR, "agent", f"{agent}.yaml"))
    cfg["task"] = _load(os.path.join(CONF_DIR, "task", f"{task}.yaml"))
    dep = deploy or defaults.get("deploy", "local")
    if dep:
        cfg = _merge(cfg, _load(os.path.join(CONF_DIR, "deploy", f"{dep}.yaml")))
    cfg = _merge(cfg, overrides or {})
    return Cfg.wrap(_num(cfg))
