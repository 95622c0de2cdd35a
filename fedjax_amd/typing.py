"""Type aliases (mirror of fedjax/core/typing.py:22-39)."""

from typing import Any, Mapping, Union

import torch

BatchExample = Mapping[str, torch.Tensor]
SingleExample = Mapping[str, torch.Tensor]
BatchPrediction = Union[torch.Tensor, Mapping[str, torch.Tensor]]
SinglePrediction = Union[torch.Tensor, Mapping[str, torch.Tensor]]
PyTree = Any
Params = PyTree
OptState = PyTree
PRNGKey = torch.Tensor
ClientId = bytes
