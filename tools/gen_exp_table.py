"""Generate yieldfactormodels.jl_amd/csrc/yfm_exp_table.inc: 2^(j/64) and 2^(j/4096), j = 0..63, correctly rounded
to double-double (hi = the nearest double, lo = the nearest double to the remainder), from Python's decimal module at
60 significant digits — the table of the certified kernels' dd_exp (yfm_dd.hpp)."""
from decimal import Decimal, getcontext
from pathlib import Path

getcontext().prec = 60
LN2 = Decimal(2).ln()


def split(d):
    hi = float(d)
    return hi, float(d - Decimal(hi))


def main():
    vals = [split((Decimal(j) / 64 * LN2).exp()) for j in range(64)]
    vals += [split((Decimal(j) / 4096 * LN2).exp()) for j in range(64)]
    lines = ["// yfm_exp_table.inc — 2^(j/64) and 2^(j/4096), j = 0..63, as double-double (hi, lo) pairs: the table of",
             "// dd_exp (yfm_dd.hpp).  Generated with Python's decimal module at 60 digits (tools/gen_exp_table.py).",
             "// clang-format off"]
    lines += [f"  {{{h!r}, {lo!r}}}," for h, lo in vals]
    out = Path(__file__).resolve().parents[1] / "yieldfactormodels.jl_amd" / "csrc" / "yfm_exp_table.inc"
    out.write_text("\n".join(lines) + "\n// clang-format on\n")


if __name__ == "__main__":
    main()
