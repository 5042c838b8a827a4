"""Per-kernel PMC table from tools/pmc_json.py output.

Columns: dispatches; HBM MB per dispatch (FETCH_SIZE x2 + WRITE_SIZE, the
gfx950 correction of MI355X_MICROARCH.md); write MB; VALU instructions per
MFMA; LDS bank conflicts as % of LDS-array cycles; SQ_WAIT_INST_ANY /
SQ_ACTIVE_INST_ANY; MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES over (GRBM_GUI_ACTIVE
/ 8 XCDs) x 1024 SIMDs -- the share of the dispatch's SIMD-cycles the matrix
pipes were busy (the profiler's own per-dispatch cost inflates the
denominator, so it is a lower bound).

usage: python tools/pmc_table.py <pmc.json> [substring ...]
"""
import json
import sys


def main():
    d = json.load(open(sys.argv[1]))["kernels"]
    keys = sys.argv[2:]
    rows = []
    for name, e in d.items():
        if keys and not any(k in name for k in keys):
            continue
        c = e["counters"]
        g = lambda k: c.get(k)   # noqa: E731
        hbm = e.get("hbm_bytes")
        wr = e.get("write_bytes")
        mf = g("SQ_INSTS_MFMA")
        valu = g("SQ_INSTS_VALU")
        lds = g("SQ_LDS_IDX_ACTIVE")
        bank = g("SQ_LDS_BANK_CONFLICT")
        wia, aia = g("SQ_WAIT_INST_ANY"), g("SQ_ACTIVE_INST_ANY")
        busy, gui = g("SQ_VALU_MFMA_BUSY_CYCLES"), g("GRBM_GUI_ACTIVE")
        f = lambda v, fmt: (fmt % v) if v is not None else "-"   # noqa: E731
        rows.append((hbm or 0, "%s | %d | %s | %s | %s | %s | %s | %s" % (
            name.split("(")[0].replace("void ", ""), e["dispatches"],
            f(hbm / 1e6 if hbm else None, "%.2f"), f(wr / 1e6 if wr else None, "%.2f"),
            f(valu / mf if valu is not None and mf else None, "%.2f"),
            f(100.0 * bank / lds if bank is not None and lds else None, "%.2f"),
            f(wia / aia if wia is not None and aia else None, "%.2f"),
            f(100.0 * busy / (gui / 8.0 * 1024) if busy is not None and gui else None, "%.1f"))))
    print("kernel | dispatches | HBM MB (FETCHx2+WRITE) | write MB | VALU/MFMA | LDS bank % | "
          "WAIT_INST/ACTIVE | MFMA busy %")
    for _, r in sorted(rows, key=lambda t: -t[0]):
        print(r)


if __name__ == "__main__":
    main()
