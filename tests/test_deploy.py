"""Deploy artefacts stay consistent with the code (reference analogue: the
`helm lint` job in .github/workflows/ci.yaml and the hand-written CRD YAML).

* every example manifest passes the same validation the admission webhook runs;
* rendered CRDs under the chart equal what kgwe/api/crds.py renders now;
* every .Values.* path used by a template exists in values.yaml;
* every metric the dashboard / PrometheusRule queries is exported by the
  native metric registry;
* the controller ConfigMap only sets keys the controller accepts.
"""
from __future__ import annotations

import json
import re
from pathlib import Path

import pytest
import yaml

from kgwe.api import crds

ROOT = Path(__file__).resolve().parents[1]
CHART = ROOT / "deploy" / "helm" / "kgwe-mi355x"


def _docs(path: Path):
    return [d for d in yaml.safe_load_all(path.read_text()) if d]


@pytest.mark.parametrize("path", sorted((ROOT / "examples").glob("*.yaml")), ids=lambda p: p.name)
def test_examples_validate(path):
    for doc in _docs(path):
        assert doc["apiVersion"] == f"{crds.GROUP}/{crds.VERSION}"
        obj = crds.default(doc)
        assert crds.validate(obj) == [], (path.name, doc["metadata"]["name"])


def test_rendered_crds_up_to_date(tmp_path):
    crds.render(tmp_path)
    for p in tmp_path.iterdir():
        assert (CHART / "crds" / p.name).read_text() == p.read_text(), p.name


def _values_paths(d: dict, prefix=()):
    for k, v in d.items():
        yield prefix + (k,)
        if isinstance(v, dict):
            yield from _values_paths(v, prefix + (k,))


def test_template_values_exist():
    values = yaml.safe_load((CHART / "values.yaml").read_text())
    have = {".".join(p) for p in _values_paths(values)}
    used = set()
    for t in (CHART / "templates").glob("*"):
        used |= set(re.findall(r"\.Values\.([A-Za-z0-9_.]+)", t.read_text()))
    missing = sorted(u for u in used if u not in have)
    assert not missing, missing


def _queried_metrics() -> set[str]:
    names = set()
    dash = json.loads((ROOT / "deploy" / "monitoring" / "grafana-dashboard.json").read_text())
    for p in dash["panels"]:
        for t in p.get("targets", []):
            names |= set(re.findall(r"\bkgwe_[a-z0-9_]+", t["expr"]))
    names |= set(re.findall(r"\bkgwe_[a-z0-9_]+", (CHART / "templates" / "monitoring.yaml").read_text()))
    return {re.sub(r"_(bucket|sum|count)$", "", n) if n.startswith("kgwe_scheduling_latency") else n
            for n in names}


def test_dashboard_matches_exported_metrics():
    from kgwe import core

    plat = core.Platform({})
    plat.add_fake_node(core.make_fixture("n0", 8, 2))
    text = plat.expose_metrics()
    declared = set(re.findall(r"^# TYPE (kgwe_[a-z0-9_]+)", text, re.M))
    missing = sorted(_queried_metrics() - declared)
    assert not missing, missing


def test_dashboard_generator_is_deterministic():
    import importlib.util

    spec = importlib.util.spec_from_file_location("gen", ROOT / "deploy" / "monitoring" / "gen_dashboard.py")
    gen = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(gen)
    want = json.dumps(gen.build(), indent=2) + "\n"
    for out in gen.OUTPUTS:
        assert Path(out).read_text() == want


def test_controller_configmap_keys_accepted():
    from kgwe.controller.main import DEFAULTS

    text = (CHART / "templates" / "controller.yaml").read_text()
    block = text.split("controller.yaml: |", 1)[1].split("---", 1)[0]
    top = set(re.findall(r"^    ([A-Za-z]+):", block, re.M))
    assert top <= set(DEFAULTS), top - set(DEFAULTS)
    values = yaml.safe_load((CHART / "values.yaml").read_text())
    assert set(values["controller"]["scheduler"]) <= set(DEFAULTS["scheduler"])
    assert set(values["controller"]["cost"]) <= set(DEFAULTS["cost"])
