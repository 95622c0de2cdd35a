"""Aggregators (mirror of fedjax/aggregators/__init__.py for the mean path)."""

from fedjax_amd.aggregators.aggregator import Aggregator
from fedjax_amd.aggregators.aggregator import AggregatorState
from fedjax_amd.aggregators.aggregator import MeanAggregatorState
from fedjax_amd.aggregators.aggregator import mean_aggregator
from fedjax_amd.aggregators.streaming import RunningMean
from fedjax_amd.aggregators import compression
from fedjax_amd.aggregators import walsh_hadamard
from fedjax_amd.aggregators.compression import rotated_uniform_stochastic_quantizer
from fedjax_amd.aggregators.compression import structured_drive_quantizer
from fedjax_amd.aggregators.compression import terngrad_quantizer
from fedjax_amd.aggregators.compression import uniform_stochastic_quantizer
# the reference's re-exports (fedjax/aggregators/__init__.py)
from fedjax_amd.aggregators.compression import binary_stochastic_quantize
from fedjax_amd.aggregators.compression import uniform_stochastic_quantize
from fedjax_amd.aggregators.compression import uniform_stochastic_quantize_pytree
from fedjax_amd.aggregators.walsh_hadamard import walsh_hadamard_transform
