"""The generated widget / API reference (tools/make_docs.py) covers every widget and every
public estimator, and the committed doc/ pages exist for them."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import make_docs  # noqa: E402


def test_every_widget_documented():
    ws = make_docs.widget_classes()
    assert len(ws) >= 27                       # 14 data + 8 ML reference widgets + additions
    for cat, mod, cls in ws:
        page = make_docs.widget_page(cat, mod, cls)
        assert page.startswith(f"# {cls.name}")
        assert os.path.exists(os.path.join(ROOT, "doc", "widgets", make_docs.slug(cls.name) + ".md")), cls.name


def test_api_pages_list_params():
    page = make_docs.api_page("classification")
    for name in ("LogisticRegression", "GBTClassifier", "LinearSVC"):
        assert f"## {name}" in page
    assert "| `regParam` |" in page
