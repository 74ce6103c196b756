"""Compare the HIP path (any SGUFP_LIB_PATH / SGUFP_CUT_BATCH) with the golden fixtures.

    python tools/ab_check.py [case ...] --cb 1,4,8,16

Debug aid: prints the first mismatches per case and batch size."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("cases", nargs="*")
    ap.add_argument("--cb", default="1,4,8,16")
    args = ap.parse_args()
    import golden_io
    from sgufp_solver_amd import engine as E
    from sgufp_solver_amd import pools
    cases = golden_io.manifest()
    if args.cases:
        cases = [c for c in cases if c["name"] in args.cases]
    for cb in args.cb.split(","):
        os.environ["SGUFP_CUT_BATCH"] = cb
        for case in cases:
            d = golden_io.case_dir(case["name"])
            e = E.Engine(f"{d}/net.txt", 0, 256)
            e.add_cuts(pools.read_pool(f"{d}/cuts.txt"))
            nodes = pools.read_nodes(f"{d}/nodes.txt")
            for run in case["runs"]:
                got = e.relax(nodes, float.fromhex(run["incumbent"]))
                want = golden_io.parse_results_text(golden_io.read_golden(case["name"], run["file"]))
                bad = golden_io.compare_results(got, want)
                print(f"cb={cb} {case['name']} {run['file']}: {'OK' if not bad else str(len(bad)) + ' bad'}")
                for b in bad[:5]:
                    print("   ", b)
            e.close()


if __name__ == "__main__":
    main()
