"""fedjax_amd — MI355X-native FedJAX server-side client-update aggregation.

Public surface mirrors the part of ``fedjax`` the aggregation path uses:
``fedjax_amd.tree_util`` (fedjax/core/tree_util.py), ``fedjax_amd.aggregators``
(fedjax/aggregators/aggregator.py), ``fedjax_amd.dataclass``
(fedjax/core/dataclasses.py) and the typing aliases. The arithmetic runs in the
HIP kernels of ``libfjagg.so`` (C ABI: include/fjagg.h).
"""

from fedjax_amd import aggregators
from fedjax_amd import random
from fedjax_amd import server
from fedjax_amd import tree_util
from fedjax_amd.dataclasses import dataclass
from fedjax_amd.slab import ClientDeltaSlab
from fedjax_amd.typing import ClientId, OptState, Params, PRNGKey, PyTree

__version__ = "0.1.0"
