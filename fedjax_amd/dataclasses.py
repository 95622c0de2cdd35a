"""Frozen dataclasses that are pytrees (mirror of fedjax/core/dataclasses.py:23-53).

``Aggregator``, ``MeanAggregatorState`` and algorithm server states are declared
with this decorator in the reference; fields whose metadata says
``pytree_node=False`` are structure (aux data), the rest are children.
"""

from __future__ import annotations

import dataclasses

from fedjax_amd import pytree


def dataclass(clz: type):
    """Creates a frozen dataclass registered as a pytree node."""
    data_clz = dataclasses.dataclass(frozen=True)(clz)
    meta_fields, data_fields = [], []
    for name, field_info in data_clz.__dataclass_fields__.items():
        if field_info.metadata.get("pytree_node", True):
            data_fields.append(name)
        else:
            meta_fields.append(name)

    def replace(self, **updates):
        """Returns a new object replacing the specified fields with new values."""
        return dataclasses.replace(self, **updates)

    data_clz.replace = replace

    def flatten_fn(x):
        return (tuple(getattr(x, n) for n in data_fields),
                tuple(getattr(x, n) for n in meta_fields))

    def unflatten_fn(meta, data):
        return data_clz(**dict(zip(meta_fields, meta)), **dict(zip(data_fields, data)))

    pytree.register_pytree_node(data_clz, flatten_fn, unflatten_fn)
    return data_clz
