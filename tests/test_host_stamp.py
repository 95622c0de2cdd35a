"""_fjhost.so reaches into torch's TensorImpl / THPVariable layout, so it must run under the
torch it was compiled against. build() writes the torch stamp into the
library (TORCH_STAMP) and into a file beside it; _lib.host() checks the file before it loads
the library and the compiled-in stamp after. A doctored or missing stamp file gets a clear
error, not a load attempt."""
import os
import shutil

import pytest

from fedjax_amd import _lib


def test_the_loaded_extension_carries_this_torch_stamp():
    h = _lib.host()
    assert h.TORCH_STAMP == _lib.torch_stamp()
    with open(_lib.host_stamp_path()) as f:
        assert f.read().strip() == _lib.torch_stamp()
    assert _lib.torch_stamp().startswith("torch ")


@pytest.mark.parametrize("stamp", ["torch 9.9.9 git deadbeef hip 0.0 cxx11abi 1 py 3.10", None])
def test_a_doctored_or_missing_stamp_is_refused_before_loading(tmp_path, monkeypatch, stamp):
    so = tmp_path / "_fjhost.so"
    shutil.copy(_lib.HOST_PATH, so)
    if stamp is not None:
        (tmp_path / "_fjhost.so.torch").write_text(stamp + "\n")
    monkeypatch.setattr(_lib, "HOST_PATH", str(so))
    monkeypatch.setattr(_lib, "_host", None)
    want = "torch 9.9.9" if stamp else "no stamp file"
    with pytest.raises(_lib.FjaggError, match=f"built against \\[{want}.*this process runs \\[torch .*rebuild"):
        _lib.host()
    assert os.path.exists(so)  # nothing was rebuilt or removed behind the caller's back
