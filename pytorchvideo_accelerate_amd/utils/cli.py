"""Fire-compatible command-line parsing (``fire`` is not installed; reference ``run.py:424-427``).

Every keyword argument of the target function becomes a flag, with Fire's value semantics
(SURVEY.md D27 / Appendix A):

* ``--name value`` and ``--name=value``; ``-`` and ``_`` are interchangeable in names;
* ``--flag`` alone means ``True`` for a boolean; ``--noflag`` means ``False``;
* values are Python-literal-evaluated (``1000`` → int, ``0.1`` → float, ``None``, ``[1,2]``), falling
  back to the raw string — so ``--checkpointing_steps 1000`` yields the *int* 1000, exactly as Fire
  (which is what silently disabled step checkpointing in the reference, R7a; our trainer accepts it).
* positional arguments fill the parameters in order.
"""
from __future__ import annotations

import ast
import inspect
from typing import Any, Callable, Dict, List, Optional, Sequence


def _literal(v: str) -> Any:
    try:
        return ast.literal_eval(v)
    except (ValueError, SyntaxError):
        low = v.lower()
        if low in ("true", "false"):
            return low == "true"
        if low == "none":
            return None
        return v


def parse_fire_args(fn: Callable, argv: Sequence[str]) -> Dict[str, Any]:
    sig = inspect.signature(fn)
    params = [p for p in sig.parameters.values() if p.kind in (p.POSITIONAL_OR_KEYWORD, p.KEYWORD_ONLY)]
    names = {p.name for p in params}
    bools = {p.name for p in params if isinstance(p.default, bool)}
    out: Dict[str, Any] = {}
    positional: List[Any] = []
    i = 0
    argv = list(argv)
    while i < len(argv):
        a = argv[i]
        if a.startswith("--") and len(a) > 2:
            body = a[2:]
            if "=" in body:
                k, v = body.split("=", 1)
                k = k.replace("-", "_")
                if k not in names:
                    raise SystemExit(f"unknown flag --{k}")
                out[k] = _literal(v)
                i += 1
                continue
            k = body.replace("-", "_")
            if k not in names and k.startswith("no") and k[2:] in bools:
                out[k[2:]] = False
                i += 1
                continue
            if k not in names:
                raise SystemExit(f"unknown flag --{k}")
            nxt = argv[i + 1] if i + 1 < len(argv) else None
            if k in bools and (nxt is None or nxt.startswith("--") or nxt.lower() not in ("true", "false")):
                out[k] = True
                i += 1
                continue
            if nxt is None:
                if k in bools:
                    out[k] = True
                    i += 1
                    continue
                raise SystemExit(f"flag --{k} needs a value")
            out[k] = _literal(nxt)
            i += 2
        else:
            positional.append(_literal(a))
            i += 1
    for p, v in zip([p for p in params if p.name not in out], positional):
        out[p.name] = v
    return out


def fire_main(fn: Callable, argv: Optional[Sequence[str]] = None):
    import sys
    argv = sys.argv[1:] if argv is None else argv
    if argv and argv[0] in ("-h", "--help"):
        print(inspect.getdoc(fn) or fn.__name__)
        print("\nFlags:")
        for p in inspect.signature(fn).parameters.values():
            print(f"  --{p.name} (default {p.default!r})")
        return None
    return fn(**parse_fire_args(fn, argv))
