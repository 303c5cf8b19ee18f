"""Minimal Hydra-compatible config composer for configurations/*.yaml.

The reference drives everything through `@hydra.main(config_path="configurations",
config_name="config")` (main.py:32) with CLI overrides `group=option` and `a.b.c=value`
(scripts/*.sh). hydra-core and omegaconf are not installed here, so this module implements
the subset the reference uses: a `defaults` list with `_self_`, group selection, dotted
overrides with Hydra's value grammar (ints, floats incl. `1e-2`, bools, null, strings), and
attribute access (`cfg.pde_instance.domain_dim`).
"""
from __future__ import annotations

import copy
import os
from typing import Any, Iterable

import yaml

CONFIG_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "configurations")


class DictConfig(dict):
    """dict with attribute access, like omegaconf.DictConfig for the keys the code reads."""

    def __getattr__(self, key):
        try:
            return self[key]
        except KeyError as e:
            raise AttributeError(key) from e

    def __setattr__(self, key, value):
        self[key] = value

    def __deepcopy__(self, memo):
        return DictConfig({k: copy.deepcopy(v, memo) for k, v in self.items()})

    def get(self, key, default=None):  # noqa: D401 - dict API
        return dict.get(self, key, default)

    def select(self, dotted: str, default=None):
        node = self
        for part in dotted.split("."):
            if not isinstance(node, dict) or part not in node:
                return default
            node = node[part]
        return node


def _wrap(obj):
    if isinstance(obj, dict):
        return DictConfig({k: _wrap(v) for k, v in obj.items()})
    if isinstance(obj, list):
        return [_wrap(v) for v in obj]
    return obj


def to_container(cfg):
    if isinstance(cfg, dict):
        return {k: to_container(v) for k, v in cfg.items()}
    if isinstance(cfg, list):
        return [to_container(v) for v in cfg]
    return cfg


def _merge(dst: dict, src: dict) -> dict:
    for k, v in src.items():
        if isinstance(v, dict) and isinstance(dst.get(k), dict):
            _merge(dst[k], v)
        else:
            dst[k] = copy.deepcopy(v)
    return dst


def parse_value(text: str) -> Any:
    """Hydra override grammar for scalars (floats like 1e-2 are floats, not strings)."""
    t = text.strip()
    low = t.lower()
    if low in ("true", "false"):
        return low == "true"
    if low in ("null", "~"):
        return None
    for cast in (int, float):
        try:
            return cast(t)
        except ValueError:
            pass
    if len(t) >= 2 and t[0] == t[-1] and t[0] in "'\"":
        return t[1:-1]
    if t.startswith("[") and t.endswith("]"):
        return yaml.safe_load(t)
    return t


def _load_yaml(path: str) -> dict:
    with open(path) as f:
        return yaml.safe_load(f) or {}


def groups(config_dir: str = CONFIG_DIR) -> list:
    return sorted(d for d in os.listdir(config_dir) if os.path.isdir(os.path.join(config_dir, d)))


def compose(config_name: str = "config", overrides: Iterable[str] = (), config_dir: str = CONFIG_DIR):
    """Compose `config_name`.yaml with its defaults list and the CLI overrides."""
    overrides = list(overrides)
    primary = _load_yaml(os.path.join(config_dir, f"{config_name}.yaml"))
    defaults = primary.pop("defaults", ["_self_"])
    group_names = set(groups(config_dir))
    choice = {}
    order = []
    for entry in defaults:
        if isinstance(entry, dict):
            (g, opt), = entry.items()
            choice[g] = opt
            order.append(g)
        else:
            order.append(entry)
    dotted = []
    for ov in overrides:
        if "=" not in ov:
            raise ValueError(f"override '{ov}' is not key=value")
        key, val = ov.split("=", 1)
        key = key.lstrip("+")
        if key in group_names and "." not in key:
            if not os.path.exists(os.path.join(config_dir, key, f"{val}.yaml")):
                raise ValueError(f"unknown option '{val}' for config group '{key}'")
            choice[key] = val
            if key not in order:
                order.insert(0, key)
        else:
            dotted.append((key, parse_value(val)))
    cfg: dict = {}
    for item in order:
        if item == "_self_":
            _merge(cfg, primary)
        else:
            _merge(cfg, {item: _load_yaml(os.path.join(config_dir, item, f"{choice[item]}.yaml"))})
    for key, val in dotted:
        node = cfg
        parts = key.split(".")
        for p in parts[:-1]:
            node = node.setdefault(p, {})
        node[parts[-1]] = val
    return _wrap(cfg)
