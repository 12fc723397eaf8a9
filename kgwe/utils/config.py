"""Config system: defaults <- YAML file <- environment <- --set flags.

Reference: Go `Default*Config()` constructors mirrored by Helm values, many
of whose keys were never read.  Here every binary
declares its full default tree; a key that is not in the tree is REJECTED
(no silently ignored settings), and values are coerced to the default's type.

* YAML: ``yaml.safe_load`` only.
* env: ``<PREFIX>A__B=value`` sets a.b (double underscore = nesting).
* flags: ``--set a.b=value``.
"""
from __future__ import annotations

import copy
import json
import os

import yaml


class ConfigError(ValueError):
    pass


def _coerce(default, value, path):
    if isinstance(default, bool):
        if isinstance(value, bool):
            return value
        if str(value).lower() in ("1", "true", "yes", "on"):
            return True
        if str(value).lower() in ("0", "false", "no", "off"):
            return False
        raise ConfigError(f"{path}: expected boolean, got {value!r}")
    if isinstance(default, int) and not isinstance(default, bool):
        try:
            return int(value)
        except (TypeError, ValueError):
            raise ConfigError(f"{path}: expected integer, got {value!r}") from None
    if isinstance(default, float):
        try:
            return float(value)
        except (TypeError, ValueError):
            raise ConfigError(f"{path}: expected number, got {value!r}") from None
    if isinstance(default, (list, dict)) and isinstance(value, str):
        try:
            return json.loads(value)
        except json.JSONDecodeError:
            raise ConfigError(f"{path}: expected JSON {type(default).__name__}") from None
    if isinstance(default, str):
        return str(value)
    return value


def _merge(base: dict, over: dict, path: str = "") -> dict:
    for k, v in over.items():
        p = f"{path}.{k}" if path else k
        if k not in base:
            raise ConfigError(f"unknown config key {p!r}")
        if isinstance(base[k], dict) and isinstance(v, dict) and base[k]:
            _merge(base[k], v, p)
        else:
            base[k] = _coerce(base[k], v, p)
    return base


def _set_path(cfg: dict, dotted: str, value: str):
    parts = dotted.split(".")
    cur = cfg
    for i, k in enumerate(parts[:-1]):
        if k not in cur or not isinstance(cur[k], dict):
            raise ConfigError(f"unknown config key {'.'.join(parts[:i + 1])!r}")
        cur = cur[k]
    if parts[-1] not in cur:
        raise ConfigError(f"unknown config key {dotted!r}")
    cur[parts[-1]] = _coerce(cur[parts[-1]], value, dotted)


def load_config(defaults: dict, path: str | None = None, sets: list[str] | None = None,
                env_prefix: str = "", environ: dict | None = None) -> dict:
    cfg = copy.deepcopy(defaults)
    if path:
        with open(path) as f:
            data = yaml.safe_load(f) or {}
        if not isinstance(data, dict):
            raise ConfigError(f"{path}: top level must be a mapping")
        _merge(cfg, data)
    env = os.environ if environ is None else environ
    if env_prefix:
        for k, v in sorted(env.items()):
            if k.startswith(env_prefix):
                dotted = ".".join(p[:1].lower() + p[1:] if p else p
                                  for p in k[len(env_prefix):].split("__"))
                _set_path(cfg, _env_key(cfg, dotted), v)
    for s in sets or []:
        if "=" not in s:
            raise ConfigError(f"--set expects key=value, got {s!r}")
        k, v = s.split("=", 1)
        _set_path(cfg, k, v)
    return cfg


def _env_key(cfg: dict, dotted: str) -> str:
    """Match env-derived keys case-insensitively against the tree."""
    cur, out = cfg, []
    for part in dotted.split("."):
        if not isinstance(cur, dict):
            raise ConfigError(f"unknown config key {dotted!r}")
        match = next((k for k in cur if k.lower() == part.lower()), None)
        if match is None:
            raise ConfigError(f"unknown config key {dotted!r}")
        out.append(match)
        cur = cur[match]
    return ".".join(out)
