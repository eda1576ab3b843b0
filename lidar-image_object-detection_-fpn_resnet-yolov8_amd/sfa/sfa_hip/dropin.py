"""Fall-through from the drop-in packages to the reference's own modules.

The reference's scripts (``test.py:14-28``, ``demo_front.py:24-37``,
``demo_2_sides.py:21-34``) append their own ``sfa`` directory to ``sys.path`` and
import a mix of hot-path modules (``models.model_utils``, ``utils.evaluation_utils``,
``utils.torch_utils``, ``data_process.kitti_bev_utils``, ``data_process.kitti_data_utils``,
``config.kitti_config``) and modules outside this build's scope
(``data_process.kitti_dataloader``, ``data_process.transformation``,
``data_process.demo_dataset``, ``utils.misc``, ``utils.visualization_utils`` …).

With the drop-in root first on ``sys.path``, ``models`` / ``utils`` / ``data_process``
/ ``config`` are this package's.  Two mechanisms keep the reference's other names
reachable, so the callers run with only their device line changed:

* every drop-in package's ``__path__`` is a :class:`FallThroughPath`: its own directory
  first, then the same sub-directory of every *reference root* — so
  ``data_process.kitti_dataloader`` (which this build does not provide) resolves to the
  reference's file, while ``data_process.kitti_bev_utils`` stays the drop-in's;
* every drop-in module that shadows a reference module ends with
  ``__getattr__ = dropin.module_getattr(__name__)``: a name the drop-in does not define
  (``kitti_data_utils.gen_hm_radius``, ``evaluation_utils._topk_channel`` …) is taken
  from the reference's module of the same dotted name, loaded once under the private
  name ``_sfa_reference.<module>`` (its own imports then bind to the drop-in's hot path).

A *reference root* is an ``sfa`` source tree of the reference (it holds
``models/fpn_resnet.py`` and ``data_process/kitti_bev_utils.py``): every
``os.pathsep``-separated entry of ``SFA_REFERENCE_ROOT``, then every such directory on
``sys.path`` other than the drop-in root.  Roots whose real path has no ancestor ending
in ``sfa`` are skipped with a warning: the reference's modules walk up from their file
until a directory name ends with ``sfa`` (``model_utils.py:16-20``,
``kitti_data_utils.py:8-12`` …) and would loop forever there.

Nothing here computes: the hot path never falls through (those names are defined by the
drop-in modules themselves and run on the HIP library).
"""

from __future__ import annotations

import importlib.util
import os
import sys
import threading
import warnings

DROPIN_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_PRIVATE = "_sfa_reference"
_lock = threading.RLock()
_roots_cache: tuple = (None, ())
_loaded: dict = {}
_warned: set = set()


def _is_reference_root(path: str) -> bool:
    return (os.path.isfile(os.path.join(path, "models", "fpn_resnet.py"))
            and os.path.isfile(os.path.join(path, "data_process", "kitti_bev_utils.py")))


def _has_sfa_ancestor(real: str) -> bool:
    p = real
    while True:
        if p.endswith("sfa"):
            return True
        parent = os.path.dirname(p)
        if parent == p:
            return False
        p = parent


def reference_roots() -> tuple:
    """Reference ``sfa`` roots, in search order (``SFA_REFERENCE_ROOT`` first)."""
    global _roots_cache
    env = os.environ.get("SFA_REFERENCE_ROOT", "")
    key = (env, tuple(sys.path))
    with _lock:
        if _roots_cache[0] == key:
            return _roots_cache[1]
        own = os.path.realpath(DROPIN_ROOT)
        roots, seen = [], {own}
        for cand in [p for p in env.split(os.pathsep) if p] + [p or os.getcwd() for p in sys.path]:
            if not isinstance(cand, str) or not os.path.isdir(cand):
                continue
            real = os.path.realpath(cand)
            if real in seen or not _is_reference_root(real):
                continue
            seen.add(real)
            if not _has_sfa_ancestor(real):
                if real not in _warned:
                    _warned.add(real)
                    warnings.warn(f"reference root {real} is not under a directory named '*sfa'; its "
                                  "modules would loop forever locating their source dir — skipped",
                                  RuntimeWarning, stacklevel=3)
                continue
            roots.append(real)
        _roots_cache = (key, tuple(roots))
        return _roots_cache[1]


class FallThroughPath:
    """A package ``__path__``: the drop-in directory, then the reference roots' ones.

    Re-evaluated at every iteration (like importlib's namespace paths), so a caller that
    appends its ``sfa`` dir to ``sys.path`` after this package was imported is still seen.
    """

    def __init__(self, own, package: str):
        self._own = list(own)
        self._rel = package.replace(".", os.sep)

    def _entries(self):
        out = list(self._own)
        for r in reference_roots():
            d = os.path.join(r, self._rel)
            if os.path.isdir(d) and d not in out:
                out.append(d)
        return out

    def __iter__(self):
        return iter(self._entries())

    def __len__(self):
        return len(self._entries())

    def __getitem__(self, i):
        return self._entries()[i]

    def __contains__(self, item):
        return item in self._entries()

    def __repr__(self):
        return f"FallThroughPath({self._entries()!r})"


def package_path(own_path, package: str) -> FallThroughPath:
    return FallThroughPath(own_path, package)


def reference_module(modname: str):
    """The reference's module ``modname`` (dotted, e.g. ``utils.evaluation_utils``),
    loaded from the first reference root holding it, or ``None``."""
    with _lock:
        if modname in _loaded:
            return _loaded[modname]
        rel = modname.replace(".", os.sep) + ".py"
        for root in reference_roots():
            path = os.path.join(root, rel)
            if not os.path.isfile(path):
                continue
            name = f"{_PRIVATE}.{modname}"
            spec = importlib.util.spec_from_file_location(name, path)
            mod = importlib.util.module_from_spec(spec)
            sys.modules[name] = mod
            try:
                spec.loader.exec_module(mod)
            except BaseException:
                sys.modules.pop(name, None)
                raise
            _loaded[modname] = mod
            return mod
        return None


def module_getattr(modname: str):
    """PEP 562 ``__getattr__`` for a drop-in module: unknown names come from the reference."""

    def __getattr__(name: str):
        if name.startswith("__"):
            raise AttributeError(name)
        ref = reference_module(modname)
        if ref is not None and hasattr(ref, name):
            return getattr(ref, name)
        raise AttributeError(
            f"module {modname!r} has no attribute {name!r}: the gfx950 drop-in does not provide it"
            + ("" if ref is not None else
               " and no reference root was found (put the reference's sfa dir on sys.path or set "
               "SFA_REFERENCE_ROOT)"))

    return __getattr__
