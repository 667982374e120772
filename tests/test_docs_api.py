"""docs/API.md stays true: its code blocks run as written (the model / operator blocks on
the CPU here, every block in order on an MI355X)."""
import re
from pathlib import Path

import pytest

DOC = Path(__file__).resolve().parents[1] / "docs" / "API.md"


def _blocks():
    return re.findall(r"```python\n(.*?)```", DOC.read_text(), re.S)


def test_api_doc_cpu_blocks_run(tmp_path, monkeypatch):
    monkeypatch.chdir(Path(__file__).resolve().parents[1])
    b = _blocks()
    assert len(b) == 4
    ns = {}
    exec(b[0].replace('"mlp.safetensors"', repr(str(tmp_path / "m.safetensors"))), ns)   # models
    exec(b[3], ns)                                                                        # operator
    assert ns["manifests"] and ns["m"].kind == "mlp"


@pytest.mark.gpu
def test_api_doc_gpu_blocks_run(gpu, tmp_path, monkeypatch):
    monkeypatch.chdir(Path(__file__).resolve().parents[1])
    b = _blocks()
    ns = {}
    exec(b[0].replace('"mlp.safetensors"', repr(str(tmp_path / "m.safetensors"))), ns)
    exec(b[1], ns)
    assert ns["st"].rows == 100 * 4096 and ns["proba"].shape == (1000,)
    exec(b[2], ns)
    assert ns["dm"].row_format == "g20" and ns["mine"]
