"""Generates the powf tables of restir-embree_amd/csrc/rs_libm.h (rs_lm_log_tab, rs_lm_exp2_tab).

  log: for m in [1 + i/128, 1 + (i+1)/128): c_i = 1 / (1 + (i + 0.5) / 128) rounded to 21 significant bits (so
       m * c_i - 1 is exact for a 24-bit m), and -log(c_i) correctly rounded to double;
  exp: 2^(j / 128), correctly rounded to double.
Values via decimal at 50 digits, printed as C99 hex floats.

  python scripts/gen_libm_tables.py
"""
from decimal import Decimal, getcontext

getcontext().prec = 50


def hexd(v):
    return float(v).hex()


def main():
    log_tab = []
    for i in range(128):
        center = Decimal(1) + (Decimal(i) + Decimal("0.5")) / 128
        c = float(round((Decimal(2) ** 20) / center)) / 2 ** 20
        assert (1 / float(center) - c) < 2 ** -19
        log_tab += [hexd(c), hexd(-Decimal(c).ln())]
    exp_tab = [hexd(Decimal(2) ** (Decimal(j) / 128)) for j in range(128)]

    def block(name, vals, per):
        lines = [", ".join(vals[k:k + per]) for k in range(0, len(vals), per)]
        return f"#define {name} {{ \\\n    " + ", \\\n    ".join(lines) + " }\n"

    print(block("RS_LM_LOG_TAB_INIT", log_tab, 4) + block("RS_LM_EXP2_TAB_INIT", exp_tab, 4))


if __name__ == "__main__":
    main()
