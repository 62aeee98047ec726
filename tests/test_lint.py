"""The tree stays lint-clean (scripts/lint.py: the reference's `.lintrunner.toml` checks that this
image can run without third-party linters)."""

import importlib.util
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _lint():
    spec = importlib.util.spec_from_file_location("ddlb_lint", os.path.join(ROOT, "scripts", "lint.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_tree_is_lint_clean(capsys):
    assert _lint().main([]) == 0, capsys.readouterr().out


def test_lint_catches_findings(tmp_path, capsys):
    bad = tmp_path / "bad.py"
    bad.write_text("import os\nimport sys\n\ntry:\n    x = 1 \nexcept:\n    pass\nprint(sys)")
    assert _lint().main([str(bad)]) == 1
    out = capsys.readouterr().out
    for msg in ("unused import 'os'", "trailing whitespace", "bare except", "missing final newline"):
        assert msg in out
    assert "unused import 'sys'" not in out
