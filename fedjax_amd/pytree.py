"""Minimal pytree flattening with ``jax.tree_util``'s leaf order.

The reference relies on ``jax.tree_util`` (a third-party dependency, SURVEY.md
§8a row A11) to walk parameter trees. This module restates the part of it the
aggregation path needs, over trees whose leaves are tensors / arrays / scalars:

* ``dict``: children in **sorted key order** (jax sorts dict keys);
* ``collections.OrderedDict`` / ``defaultdict``: insertion order / sorted order,
  as jax registers them;
* ``list``, ``tuple``, ``namedtuple``: positional;
* ``None``: an empty subtree (no leaves);
* classes registered with :func:`register_pytree_node` (``fedjax_amd.dataclass``
  registers its data fields, fedjax/core/dataclasses.py:23-53);
* anything else is a leaf.

Structure mismatches raise ``ValueError`` (``jax.tree.map`` does too).
"""

from __future__ import annotations

import collections
from typing import Any, Callable, Dict, List, Tuple

_REGISTRY: Dict[type, Tuple[Callable, Callable]] = {}
# lazy values (tree_util.WeightedTree): type -> fn(x) returning the pytree they stand for;
# every walk here materializes them where they appear
_LAZY: Dict[type, Callable] = {}


def register_lazy_type(cls: type, materialize: Callable) -> None:
    """Instances of ``cls`` stand for the pytree ``materialize(x)`` returns."""
    _LAZY[cls] = materialize


def register_pytree_node(cls: type, flatten_fn: Callable, unflatten_fn: Callable) -> None:
    """flatten_fn(x) -> (children, aux); unflatten_fn(aux, children) -> x."""
    _REGISTRY[cls] = (flatten_fn, unflatten_fn)
    _LEAF_TYPES.discard(cls)


def register_leaf_type(cls: type) -> None:
    """Declare ``cls`` a leaf type (skips the container checks in flatten_as)."""
    if cls not in _REGISTRY:
        _LEAF_TYPES.add(cls)


class TreeDef:
    """Hashable structure of a pytree (node kind, aux data, children)."""

    __slots__ = ("kind", "aux", "children", "leafy", "_hash", "_fast")

    def __init__(self, kind, aux, children):
        self.kind = kind
        self.aux = aux
        self.children = children
        # every child is a leaf: flatten_as can take the values without recursing
        self.leafy = bool(children) and all(c.kind == "leaf" for c in children)
        self._hash = None
        self._fast = False  # compiled leaf accessor (None: not compilable), see _compile

    @property
    def num_leaves(self):
        return 1 if self.kind == "leaf" else sum(c.num_leaves for c in self.children)

    def _key(self):
        return (self.kind, self.aux, self.children)

    def __eq__(self, other):
        return isinstance(other, TreeDef) and (self is other or self._key() == other._key())

    def __hash__(self):
        if self._hash is None:
            self._hash = hash(self._key())
        return self._hash

    def __repr__(self):
        if self.kind == "leaf":
            return "*"
        return f"{self.kind}{'' if self.aux is None else self.aux!r}({', '.join(map(repr, self.children))})"


_LEAF = TreeDef("leaf", None, ())
_LEAF_TYPES = set()  # types known to be leaves (fast path); filled by register_leaf_type
_NONE = TreeDef("none", None, ())


def _is_namedtuple(x) -> bool:
    return isinstance(x, tuple) and hasattr(type(x), "_fields")


def _node(tree) -> Tuple[str, Any, List[Any]]:
    """(kind, aux, children) of one node, or ('leaf', None, []) for a leaf."""
    t = type(tree)
    if tree is None:
        return "none", None, []
    if t in _REGISTRY:
        children, aux = _REGISTRY[t][0](tree)
        return "custom", (t, aux), list(children)
    if t is dict or t is collections.defaultdict:
        keys = tuple(sorted(tree))
        aux = keys if t is dict else (keys, tree.default_factory)
        return ("dict" if t is dict else "defaultdict"), aux, [tree[k] for k in keys]
    if t is collections.OrderedDict:
        keys = tuple(tree)
        return "odict", keys, [tree[k] for k in keys]
    if t is list:
        return "list", len(tree), list(tree)
    if t is tuple:
        return "tuple", len(tree), list(tree)
    if _is_namedtuple(tree):
        return "namedtuple", t, list(tree)
    return "leaf", None, []


_INTERNED = {}  # (kind, aux, children) -> TreeDef: one object per structure (capped)


def _intern(kind, aux, children) -> TreeDef:
    """The TreeDef of (kind, aux, children), shared by every flatten of that structure, so
    equality is identity and per-structure caches (compiled accessors, native specs) are
    hit without rehashing the structure. Unhashable aux data (registered classes) is not
    interned."""
    key = (kind, aux, children)
    try:
        td = _INTERNED.get(key)
    except TypeError:
        return TreeDef(kind, aux, children)
    if td is None:
        td = TreeDef(kind, aux, children)
        if len(_INTERNED) < 4096:
            _INTERNED[key] = td
    return td


def flatten(tree) -> Tuple[List[Any], TreeDef]:
    leaves: List[Any] = []
    leaf_types = _LEAF_TYPES

    def rec(x) -> TreeDef:
        if type(x) in leaf_types:  # tensors / arrays: skip the node classification
            leaves.append(x)
            return _LEAF
        if type(x) in _LAZY:
            return rec(_LAZY[type(x)](x))
        kind, aux, children = _node(x)
        if kind == "leaf":
            leaves.append(x)
            return _LEAF
        if kind == "none":
            return _NONE
        return _intern(kind, aux, tuple([rec(c) for c in children]))

    td = rec(tree)
    return leaves, td


def leaves_of(tree) -> List[Any]:
    return flatten(tree)[0]


def _is_leaf(x) -> bool:
    return type(x) in _LEAF_TYPES or _node(x)[0] == "leaf"


def flatten_as(treedef: TreeDef, tree) -> List[Any]:
    """Leaves of ``tree``, which must have structure ``treedef`` (ValueError if not).

    Walks ``treedef`` and checks ``tree`` against it node by node, without
    building a second TreeDef (this is the per-client hot loop of tree_mean)."""
    fast = treedef._fast
    if fast is False:  # first use of this TreeDef object: compiled once per structure
        fast = _FAST.get(treedef, False)
        if fast is False:
            fast = _FAST[treedef] = _compile(treedef) if len(_FAST) < 4096 else None
        treedef._fast = fast
    if fast is not None:
        leaves = fast(tree)
        if leaves is not None:
            return leaves
    out: List[Any] = []
    try:
        _collect(treedef, tree, out)
    except (KeyError, IndexError, TypeError, _Mismatch):
        raise ValueError(f"pytree structure mismatch: expected {treedef!r}, got "
                         f"{flatten(tree)[1]!r}") from None
    return out


class _Mismatch(Exception):
    pass


_FAST: Dict[TreeDef, Any] = {}  # structure -> compiled accessor (or None)


def _compile(td: TreeDef):
    """Straight-line accessor for trees of dict / list / tuple / None nodes with leaves of
    registered leaf types: returns the leaf list, or None whenever anything differs from
    ``td`` (then flatten_as takes the general walk, which also builds the error). Other
    node kinds are not compiled (returns None)."""
    lines, names = [], []
    consts: List[Any] = []  # dict keys, passed as objects (repr(key) need not be an expression)
    counter = [0]

    def var():
        counter[0] += 1
        return f"v{counter[0]}"

    def emit(t: TreeDef, ref: str) -> bool:
        k = t.kind
        if k == "leaf":
            lines.append(f"if type({ref}) not in LT: return None")
            names.append(ref)
            return True
        if k == "none":
            lines.append(f"if {ref} is not None: return None")
            return True
        if k == "dict":
            lines.append(f"if type({ref}) is not dict or len({ref}) != {len(t.aux)}: return None")
            keys = []
            for key in t.aux:
                keys.append(f"C[{len(consts)}]")
                consts.append(key)
        elif k in ("list", "tuple"):
            lines.append(f"if type({ref}) is not {k} or len({ref}) != {t.aux}: return None")
            keys = [str(i) for i in range(t.aux)]
        else:
            return False
        for key, c in zip(keys, t.children):
            v = var()
            lines.append(f"{v} = {ref}[{key}]")
            if not emit(c, v):
                return False
        return True

    try:
        if not emit(td, "x"):
            return None
        body = "\n    ".join(lines + [f"return [{', '.join(names)}]"])
        src = f"def fast(x):\n  try:\n    {body}\n  except (KeyError, IndexError, TypeError):\n    return None\n"
        ns = {"LT": _LEAF_TYPES, "C": tuple(consts)}
        exec(compile(src, f"<pytree accessor {len(names)} leaves>", "exec"), ns)  # noqa: S102 - generated
        return ns["fast"]
    except (SyntaxError, RecursionError, ValueError):
        return None


_SPECS: Dict[TreeDef, Any] = {}  # structure -> native walk spec (or None)
_SPEC_KIND = {"dict": 2, "list": 3, "tuple": 4}


def native_spec(td: TreeDef):
    """Walk program of ``td`` for fjhost.gather_rows (fedjax_amd/csrc/fjhost.cpp): 0 =
    leaf, 1 = None, ``(2, keys, children)`` dict (keys in flatten order), ``(3|4, n,
    children)`` list / tuple. None when ``td`` holds another node kind (namedtuple,
    OrderedDict, registered classes): those trees take the Python walk."""
    spec = _SPECS.get(td, False)
    if spec is False:
        spec = _SPECS[td] = _spec(td) if len(_SPECS) < 4096 else None
    return spec


def _spec(td: TreeDef):
    k = td.kind
    if k == "leaf":
        return 0
    if k == "none":
        return 1
    if k not in _SPEC_KIND:
        return None
    children = tuple(_spec(c) for c in td.children)
    if any(c is None for c in children):
        return None
    return (_SPEC_KIND[k], td.aux if k == "dict" else len(children), children)


def _collect(td: TreeDef, x, out: List[Any]) -> None:
    if type(x) in _LAZY:
        x = _LAZY[type(x)](x)
    k = td.kind
    if k == "leaf":
        if not _is_leaf(x):
            raise _Mismatch
        out.append(x)
        return
    if k == "none":
        if x is not None:
            raise _Mismatch
        return
    t = type(x)
    if k == "dict":
        if t is not dict or len(x) != len(td.aux):
            raise _Mismatch
        vals = [x[key] for key in td.aux]
    elif k in ("list", "tuple"):
        if t is not (list if k == "list" else tuple) or len(x) != td.aux:
            raise _Mismatch
        vals = x
    else:
        kind, aux, vals = _node(x)
        if kind != k or aux != td.aux or len(vals) != len(td.children):
            raise _Mismatch
    if td.leafy:
        vals = [_LAZY[type(v)](v) if type(v) in _LAZY else v for v in vals]
        for v in vals:
            if not _is_leaf(v):
                raise _Mismatch
        out.extend(vals)
        return
    for c, v in zip(td.children, vals):
        _collect(c, v, out)


def unflatten(treedef: TreeDef, leaves) -> Any:
    it = iter(leaves)

    def rec(td: TreeDef):
        k = td.kind
        if k == "leaf":
            return next(it)
        if k == "none":
            return None
        vals = [rec(c) for c in td.children]
        if k == "dict":
            return dict(zip(td.aux, vals))
        if k == "defaultdict":
            d = collections.defaultdict(td.aux[1])
            d.update(zip(td.aux[0], vals))
            return d
        if k == "odict":
            return collections.OrderedDict(zip(td.aux, vals))
        if k == "list":
            return vals
        if k == "tuple":
            return tuple(vals)
        if k == "namedtuple":
            return td.aux(*vals)
        if k == "custom":
            cls, aux = td.aux
            return _REGISTRY[cls][1](aux, vals)
        raise AssertionError(k)

    out = rec(treedef)
    if next(it, _SENTINEL) is not _SENTINEL:
        raise ValueError("too many leaves for treedef")
    return out


_SENTINEL = object()


def tree_map(fn: Callable, tree, *rest) -> Any:
    leaves, td = flatten(tree)
    others = [flatten_as(td, r) for r in rest]
    return unflatten(td, [fn(*xs) for xs in zip(leaves, *others)])
