"""INTEGRATION.md must describe the API that exists: every
``from rvs_amd... import ...`` in its python code blocks resolves, every
``rvs_amd.a.b.Name`` it names in backticks resolves, and the attributes the
pipelined-run example calls exist (the boundary document once described a
removed class)."""
import importlib
import os
import re

import pytest

DOC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "INTEGRATION.md")


def _code_blocks(text):
    return re.findall(r"```python\n(.*?)```", text, re.S)


def _imports():
    out = []
    for block in _code_blocks(open(DOC).read()):
        for line in block.splitlines():
            m = re.match(r"\s*from (rvs_amd[\w.]*) import (.+?)(#.*)?$", line)
            if m:
                for name in m.group(2).split(","):
                    out.append((m.group(1), name.split(" as ")[0].strip()))
    return out


def test_doc_has_imports():
    assert len(_imports()) >= 8


@pytest.mark.parametrize("mod,name", _imports())
def test_doc_import_resolves(mod, name):
    assert hasattr(importlib.import_module(mod), name), f"{mod}.{name} (INTEGRATION.md)"


def _dotted_names():
    names = set()
    for m in re.finditer(r"`(rvs_amd(?:\.\w+)+)", open(DOC).read()):
        names.add(m.group(1))
    return sorted(names)


@pytest.mark.parametrize("dotted", _dotted_names())
def test_doc_dotted_name_resolves(dotted):
    parts = dotted.split(".")
    obj, i = None, len(parts)
    while i > 0:  # longest importable module prefix, then attributes
        try:
            obj = importlib.import_module(".".join(parts[:i]))
            break
        except ImportError:
            i -= 1
    assert obj is not None, dotted
    for p in parts[i:]:
        assert hasattr(obj, p), f"{dotted}: no {p!r} (INTEGRATION.md)"
        obj = getattr(obj, p)


def test_pipelined_run_example_api():
    from rvs_amd.engine import RoadVisionEngine
    from rvs_amd.handback import Record
    from rvs_amd.schedule import PipelinedRun, Schedule
    import inspect
    sig = inspect.signature(RoadVisionEngine.__init__).parameters
    assert "lanes" in sig and "pair" in sig
    for attr in ("run", "wait_step", "records", "close", "step_done_ms"):
        assert hasattr(PipelinedRun, attr) or attr == "records"
    assert "units" in inspect.signature(PipelinedRun.__init__).parameters
    for attr in ("recording", "run", "close"):
        assert hasattr(Schedule, attr)
    assert hasattr(Record, "detections")
    assert not re.search(r"OverlappedSteps|graph capture", "".join(_code_blocks(open(DOC).read())))
