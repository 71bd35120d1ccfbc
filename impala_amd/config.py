"""Config tree with the reference's Hydra surface (conf/config.yaml, conf/agent/*.yaml,
conf/deploy/*.yaml, conf/task/*.yaml: the same files, keys and values; checked against the
reference's key sets by tests/test_host_logic.py), loaded with yaml.safe_load (Hydra and
OmegaConf are not dependencies): the defaults list picks the group files, ``${...}``
interpolations are resolved, attribute access works like OmegaConf (``cfg.agent.batch_size``)."""
from __future__ import annotations

import copy
import os
import re
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


_INTERP = re.compile(r"\$\{([^}]+)\}")


def _lookup(root: Dict[str, Any], path: str):
    node: Any = root
    for part in path.strip().split("."):
        if not isinstance(node, dict) or part not in node:
            raise KeyError(f"interpolation ${{{path}}}: no key {part!r}")
        node = node[part]
    return node


def _resolve(node: Any, root: Dict[str, Any], depth: int = 0):
    """OmegaConf-style ``${a.b}`` interpolation (absolute key paths): a value that is exactly one
    interpolation takes the referenced value (and type); otherwise the pieces are joined as a
    string (conf/config.yaml:17 ``${distributed.server_addr}:${distributed.m_port}``)."""
    if depth > 16:
        raise ValueError("interpolation cycle")
    if isinstance(node, dict):
        return {k: _resolve(v, root, depth) for k, v in node.items()}
    if isinstance(node, list):
        return [_resolve(v, root, depth) for v in node]
    if isinstance(node, str) and "${" in node:
        m = _INTERP.fullmatch(node)
        if m:
            return _resolve(_lookup(root, m.group(1)), root, depth + 1)
        return _INTERP.sub(lambda mm: str(_resolve(_lookup(root, mm.group(1)), root, depth + 1)),
                           node)
    return node


def _defaults(spec) -> Dict[str, str]:
    """Hydra defaults list -> {group: option}.  Accepts the reference's list form
    (``- _self_``, ``- agent: impala``, ``- override hydra/...: disabled``; the hydra logging
    overrides are ignored) and the older mapping form."""
    out: Dict[str, str] = {}
    if isinstance(spec, dict):
        return dict(spec)
    for item in spec or []:
        if isinstance(item, dict):
            for k, v in item.items():
                if not str(k).startswith("override "):
                    out[str(k)] = v
    return out


def load_config(overrides: Optional[Dict[str, Any]] = None, deploy: Optional[str] = "local",
                agent: Optional[str] = None, task: Optional[str] = None) -> Cfg:
    """Compose config.yaml + agent + task (its defaults list) + a deploy overlay (+ overrides)
    and resolve interpolations, as main.py:39-53 under ``python main.py +deploy=local``.
    ``agent`` / ``task`` select the group files as Hydra's ``agent=sac task=mujoco`` would
    (agent=sac alone implies task=mujoco, the reference's SAC task); ``deploy=None`` composes
    without an overlay."""
    base = _load(os.path.join(CONF_DIR, "config.yaml"))
    defaults = _defaults(base.pop("defaults", []))
    cfg = dict(base)
    agent = agent or defaults.get("agent", "impala")
    task = task or ("mujoco" if agent == "sac" else defaults.get("task", "procgen"))
    cfg["agent"] = _load(os.path.join(CONF_DIR, "agent", f"{agent}.yaml"))
    cfg["task"] = _load(os.path.join(CONF_DIR, "task", f"{task}.yaml"))
    dep = deploy if deploy is not None else defaults.get("deploy")
    if dep:
        cfg = _merge(cfg, _load(os.path.join(CONF_DIR, "deploy", f"{dep}.yaml")))
    cfg = _merge(cfg, overrides or {})
    return Cfg.wrap(_num(_resolve(cfg, cfg)))
