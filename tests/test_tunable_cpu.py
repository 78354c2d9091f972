"""utils/tunable.py on the CPU: where the shipped results live, that they are well-formed
TunableOp files for this stack (validator rows + GEMM rows), and that the A/B switch leaves
TunableOp untouched."""
import csv
import os

from vodascheduler_amd.utils import tunable


def test_results_path_and_override(monkeypatch, tmp_path):
    assert tunable.results_path("fp32").endswith(os.path.join("var", "tunableop", "fp32.csv"))
    monkeypatch.setenv("VODA_TUNABLEOP_DIR", str(tmp_path))
    assert tunable.results_path("bf16") == str(tmp_path / "bf16.csv")


def test_shipped_results_are_tunableop_files():
    for prec, dtype_tag in (("fp32", "float"), ("bf16", "BFloat16")):
        path = tunable.results_path(prec)
        if not os.path.exists(path):
            continue
        rows = list(csv.reader(open(path)))
        validators = {r[1]: r[2] for r in rows if r and r[0] == "Validator"}
        assert {"PT_VERSION", "HIPBLASLT_VERSION", "GCN_ARCH_NAME"} <= set(validators)
        assert validators["GCN_ARCH_NAME"].startswith("gfx950")
        gemms = [r for r in rows if r and r[0] != "Validator"]
        assert gemms and all(len(r) == 4 and float(r[3]) > 0 for r in gemms)
        assert any(dtype_tag in r[0] for r in gemms)


def test_disabled_switch_does_not_enable(monkeypatch):
    monkeypatch.setenv("VODA_TUNABLEOP", "0")
    monkeypatch.setattr(tunable, "_DONE", {})
    assert tunable.configure("fp32") is False
