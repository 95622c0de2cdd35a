"""Aggregators (mirror of fedjax/aggregators/__init__.py for the mean path)."""

from fedjax_amd.aggregators.aggregator import Aggregator
from fedjax_amd.aggregators.aggregator import AggregatorState
from fedjax_amd.aggregators.aggregator import MeanAggregatorState
from fedjax_amd.aggregators.aggregator import mean_aggregator
from fedjax_amd.aggregators.streaming import RunningMean
