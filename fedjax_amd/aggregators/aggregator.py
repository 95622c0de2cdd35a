"""Aggregator interface and the weighted-mean aggregator.

Mirror of google/fedjax 0.0.17 ``fedjax/aggregators/aggregator.py``:

* :class:`Aggregator` — frozen pytree dataclass of ``init`` / ``apply`` (:26-53);
* :class:`MeanAggregatorState` — empty state (:56-58);
* :func:`mean_aggregator` — ``apply`` lazily drops client ids and calls
  :func:`fedjax_amd.tree_util.tree_mean` (:61-75; the call at :73), which folds all K clients on
  the GPU in one kernel launch per leaf-dtype group.
"""

from typing import Any, Callable, Iterable, Tuple

from fedjax_amd import dataclasses
from fedjax_amd import tree_util
from fedjax_amd.typing import ClientId, Params

PyTree = Any
AggregatorState = PyTree


@dataclasses.dataclass
class Aggregator:
    """Interface for algorithms to aggregate (aggregator.py:26-53).

    Usage, as in the reference::

      aggregator = mean_aggregator()
      state = aggregator.init()
      for i in range(num_rounds):
        clients_params_and_weights = compute_client_outputs(i)
        aggregated_params, state = aggregator.apply(clients_params_and_weights, state)

    Attributes:
      init: Returns initial state of aggregator.
      apply: Returns the new aggregator state and aggregated params.
    """
    init: Callable[[], AggregatorState]
    apply: Callable[[Iterable[Tuple[ClientId, Params, float]], AggregatorState],
                    Tuple[Params, AggregatorState]]


@dataclasses.dataclass
class MeanAggregatorState:
    """Mean aggregator is stateless."""


def mean_aggregator() -> Aggregator:
    """Builds (weighted) mean aggregator.

    ``apply`` returns ``tree_util.tree_mean``'s result: its float32 leaves may be slices of
    one allocation (see tree_mean), so one kept leaf holds the whole mean's memory."""

    def init():
        return MeanAggregatorState()

    def apply(clients_params_and_weights, state):
        def extract_params_and_weight(clients_params_and_weight):
            _, param, weight = clients_params_and_weight
            return param, weight

        if type(clients_params_and_weights) in (list, tuple) and clients_params_and_weights:
            # resident clients: the triples go to the one-call native path as they are
            # (tree_util.mean_of_triples); a one-shot iterable keeps the lazy map and the
            # streaming fold
            return tree_util.mean_of_triples(clients_params_and_weights), state
        params_and_weights = map(extract_params_and_weight, clients_params_and_weights)
        return tree_util.tree_mean(params_and_weights), state

    return Aggregator(init, apply)
