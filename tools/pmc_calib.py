"""FETCH_SIZE / WRITE_SIZE per known byte count for each access width of tools/pmc_calib.hip.

usage: pmc_calib.py OUT_DIR  (OUT_DIR/FETCH_SIZE and OUT_DIR/WRITE_SIZE: rocprofv3 --pmc runs of build/pmc_calib)
Prints, per kernel, the counter in bytes (KiB x 1024) and the factor known_bytes / counter_bytes: the multiplier that
turns the counter into bytes moved for that access width."""
import json
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from traffic import per_dispatch  # noqa: E402

READ = 256 << 20
WRITE = 32 << 20
WIDTH = {"unsigned int": 4, "unsigned long long": 8, "HIP_vector_type<unsigned int, 4u>": 16, "uint4": 16}


def width(name: str) -> int:
    inner = name.split("<", 1)[1].rsplit(">", 1)[0] if "<" in name else ""
    for k, v in WIDTH.items():
        if inner.startswith(k):
            return v
    return 0


def main():
    root = sys.argv[1]
    fetch, fn = per_dispatch(root, "FETCH_SIZE")
    write, wn = per_dispatch(root, "WRITE_SIZE")
    out = {"method": "tools/pmc_calib.hip: each kernel reads 256 MiB once (4 / 8 / 16 B per lane, coalesced) or writes "
                     "32 MiB once; factor = known bytes / (counter KiB x 1024)", "read": {}, "write": {}}
    for d, v in fetch.items():
        name = fn[d]
        if name.startswith("void read_kernel") or name.startswith("read_kernel"):
            out["read"][f"{width(name)}B/lane"] = {"fetch_size_bytes": int(v * 1024), "factor": round(READ / (v * 1024), 3)}
    for d, v in write.items():
        name = wn[d]
        if name.startswith("void write_kernel") or name.startswith("write_kernel"):
            out["write"][f"{width(name)}B/lane"] = {"write_size_bytes": int(v * 1024), "factor": round(WRITE / (v * 1024), 3)}
    # scattered single words (the commit / select pattern): one word per 128-B line, READ / 128 lines read, WRITE / 128
    # lines written; bytes_per_line = counter bytes / lines touched, so HBM bytes = lines x bytes_per_line
    out["scattered"] = {"method": "one 4- or 8-B word per 128-B line, every line once, scrambled line order; gather1 / "
                                  "scatter1: lane 0 of each wave, gather64: every lane its own line",
                        "raw_counter_bytes_per_line": {}}
    for src, total, lines, pre in ((fetch, READ, READ // 128, ("gather1", "gather64")), (write, WRITE, WRITE // 128, ("scatter1",))):
        names = fn if src is fetch else wn
        for d, v in src.items():
            name = names[d].removeprefix("void ")
            k = next((p for p in pre if name.startswith(p + "_kernel")), None)
            if k is None:
                continue
            w = width(names[d])
            out["scattered"]["raw_counter_bytes_per_line"][f"{k}/{w}B"] = {
                "counter_bytes": int(v * 1024), "lines": lines, "counter_bytes_per_line": round(v * 1024 / lines, 2),
                "algorithmic_bytes_per_line": w}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
