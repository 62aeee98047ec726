"""Per-implementation option schema and environment guard.

Parity: ``ddlb/primitives/TPColumnwise/utils.py:9-108`` (``EnvVarGuard``, ``OptionsManager``;
the TPRowwise copy is byte-identical). Differences:

* ``(min, max)`` tuples validate *integers* for integer defaults (``s=2.5`` is rejected);
* ``ALIASES`` lets an implementation accept reference spellings (``nccl`` for RCCL) and map
  them to the native value before validation;
* ``EnvVarGuard`` restores in ``restore()`` / context-exit, not only ``__del__``.
"""

from __future__ import annotations

import os
from typing import Any, Dict, Mapping, Optional


class EnvVarGuard:
    """Set environment variables now; put the previous values back on ``restore()``."""

    def __init__(self, env_vars: Mapping[str, str]):
        self.env_vars = dict(env_vars)
        self._saved: Dict[str, Optional[str]] = {}
        for key, value in self.env_vars.items():
            self._saved[key] = os.environ.get(key)
            os.environ[key] = str(value)

    def restore(self) -> None:
        for key, old in self._saved.items():
            if old is None:
                os.environ.pop(key, None)
            else:
                os.environ[key] = old
        self._saved = {}

    def __enter__(self) -> "EnvVarGuard":
        return self

    def __exit__(self, *exc) -> None:
        self.restore()

    def __del__(self):
        try:
            self.restore()
        except Exception:
            pass


class OptionsManager:
    """Validate implementation options against ``DEFAULT_OPTIONS`` / ``ALLOWED_VALUES``."""

    #: keys the runner passes through that are not implementation options
    BENCHMARK_OPTIONS = frozenset({"implementation"})

    def __init__(self, default_options: Mapping[str, Any],
                 allowed_values: Optional[Mapping[str, Any]] = None,
                 aliases: Optional[Mapping[str, Mapping[Any, Any]]] = None):
        self.default_options = dict(default_options)
        self.allowed_values = dict(allowed_values or {})
        self.aliases = {k: dict(v) for k, v in (aliases or {}).items()}
        self.options: Dict[str, Any] = dict(self.default_options)

    def parse(self, kwargs: Mapping[str, Any]) -> None:
        opts = {k: v for k, v in kwargs.items() if k not in self.BENCHMARK_OPTIONS}
        unknown = set(opts) - set(self.default_options)
        if unknown:
            raise ValueError(f"Unknown options provided: {sorted(unknown)}. "
                             f"Valid options are: {list(self.default_options)}")
        for key, value in opts.items():
            value = self.aliases.get(key, {}).get(value, value)
            self.options[key] = value
        for key, allowed in self.allowed_values.items():
            if key not in self.options:
                continue
            value = self.options[key]
            if isinstance(allowed, tuple) and len(allowed) == 2:
                lo, hi = allowed
                is_num = isinstance(value, (int, float)) and not isinstance(value, bool)
                if isinstance(self.default_options.get(key), int) and not isinstance(
                        self.default_options.get(key), bool):
                    is_num = is_num and float(value).is_integer()
                    if is_num:
                        value = int(value)
                        self.options[key] = value
                if not (is_num and lo <= value <= hi):
                    raise ValueError(f"Invalid value for {key}: {value!r}. "
                                     f"Must be a number between {lo} and {hi}")
            elif value not in allowed:
                raise ValueError(f"Invalid value for {key}: {value!r}. Must be one of {list(allowed)}")

    def get(self, key: str, default: Any = None) -> Any:
        return self.options.get(key, default)

    def __getitem__(self, key: str) -> Any:
        return self.options[key]

    def __contains__(self, key: str) -> bool:
        return key in self.options

    def as_dict(self) -> Dict[str, Any]:
        return dict(self.options)
