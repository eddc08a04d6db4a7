"""Each kernel against every pipe it uses, from tools/pmc_pipes.sh (two --pmc passes) and the
static VALU mix of profiles/isa_mix.json -> profiles/pipes.json.

Per dispatch (each kernel's batch dispatches: grid >= 1/32 of its largest; rocprofv3 --pmc
serialises dispatches, so each is measured alone) with C = GRBM_GUI_ACTIVE / 8 the dispatch's
cycles (rocprofv3 sums the 8 XCDs) and the counters' own units (MI355X_MICROARCH.md, PMC table):
  valu_mix   SQ_INSTS_VALU x 2 / mix_roof / (1024 SIMDs x C): the VALU issue the kernel's
             instructions need at the sustained rate of its own class mix (tools/isa_mix.py),
             over the cycles the dispatch took -- its VALU fraction of its own mix peak
  lds        SQ_LDS_IDX_ACTIVE / (256 CUs x C): LDS-array busy (bank conflicts included)
  ta, td     TA_TA_BUSY_sum, TD_TD_BUSY_sum / (256 x C): texture address / data units busy
  mfma       SQ_VALU_MFMA_BUSY_CYCLES / (1024 x C)
  issue      SQ_ACTIVE_INST_ANY (quad-cycles, summed over waves) / (256 x C): wave-instruction
             activity per SIMD (several waves of a SIMD can be active on different pipes)
The binding pipe is the largest of the throughput fractions valu_mix / lds / mfma; bench.py
adds HBM (measured traffic over its live dispatch time) and labels the roofline by the largest.
TA / TD busy are reported but are not throughput roofs: they count cycles with any request in
flight, latency included -- halving orient_desc's cache accesses (r7p: 4.07e8 -> 1.81e8
TCP_TOTAL_CACHE_ACCESSES) left TD_TD_BUSY unchanged at ~0.87, and nearly every kernel reads
0.5-0.9 on them whatever its byte rate.
Usage: python tools/pipes.py gpurun_out/pipes [batch] > profiles/pipes.json"""
import collections
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PIPES = ("valu_mix", "lds", "mfma")  # throughput roofs (ta / td: occupancy, see above)


def kernel_key(name):
    n = name.replace("void ", "").replace("slamgpu::", "").replace("(anonymous namespace)::", "")
    return n.split("(")[0]


def per_dispatch(d):
    """kernel -> counter -> mean over the kernel's batch dispatches (each dispatch summed over
    its dimensions)."""
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    grid = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = kernel_key(r["Kernel_Name"])
            did = r.get("Dispatch_Id", r.get("Correlation_Id", ""))
            acc[(k, did)][r["Counter_Name"]] += float(r["Counter_Value"])
            grid[(k, did)] = int(r.get("Grid_Size", 0) or 0)
    gmax = collections.defaultdict(int)
    for (k, did), g in grid.items():
        gmax[k] = max(gmax[k], g)
    out = collections.defaultdict(lambda: collections.defaultdict(list))
    for (k, did), cs in acc.items():
        if 32 * grid[(k, did)] >= gmax[k]:
            for c, v in cs.items():
                out[k][c].append(v)
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in out.items()}


def main():
    base = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pipes"
    batch = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    mix = json.load(open(os.path.join(ROOT, "profiles", "isa_mix.json")))["kernels"]
    p1, p2 = per_dispatch(os.path.join(base, "p1")), per_dispatch(os.path.join(base, "p2"))
    res = {"batch": batch, "valu_issue_peak_per_s": 1.2288e12,
           "source": "tools/pmc_pipes.sh (bench.py --steps 2 --warmup 1, two rocprofv3 --pmc "
                     "passes) + tools/pipes.py; VALU mix roof from profiles/isa_mix.json",
           "definitions": {
               "cycles": "GRBM_GUI_ACTIVE / 8 per dispatch",
               "valu_mix": "SQ_INSTS_VALU * 2 / mix_roof / (1024 * cycles)",
               "lds": "SQ_LDS_IDX_ACTIVE / (256 * cycles)",
               "ta": "TA_TA_BUSY_sum / (256 * cycles)", "td": "TD_TD_BUSY_sum / (256 * cycles)",
               "mfma": "SQ_VALU_MFMA_BUSY_CYCLES / (1024 * cycles)",
               "issue": "SQ_ACTIVE_INST_ANY / (256 * cycles)",
               "lds_conflict_per_instr": "SQ_LDS_BANK_CONFLICT / SQ_INSTS_LDS"},
           "kernels": {}}
    for k in sorted(set(p1) & set(p2)):
        a, b = p1[k], p2[k]
        cyc = a.get("GRBM_GUI_ACTIVE", 0) / 8.0
        if cyc <= 0 or a.get("SQ_WAVES", 0) <= 0:
            continue
        m = mix.get(k)
        ent = {"cycles_per_dispatch": round(cyc),
               "sq_insts_valu_per_dispatch": a.get("SQ_INSTS_VALU"),
               "sq_insts_salu_per_dispatch": a.get("SQ_INSTS_SALU"),
               "sq_insts_lds_per_dispatch": a.get("SQ_INSTS_LDS"),
               "sq_insts_vmem_per_dispatch": a.get("SQ_INSTS_VMEM"),
               "sq_insts_smem_per_dispatch": b.get("SQ_INSTS_SMEM"),
               "sq_waves_per_dispatch": a.get("SQ_WAVES"),
               "tcp_cache_accesses_per_dispatch": b.get("TCP_TOTAL_CACHE_ACCESSES_sum"),
               "tcp_tcc_read_req_per_dispatch": b.get("TCP_TCC_READ_REQ_sum")}
        fr = {"lds": b.get("SQ_LDS_IDX_ACTIVE", 0) / (256 * cyc),
              "ta": a.get("TA_TA_BUSY_sum", 0) / (256 * cyc),
              "td": a.get("TD_TD_BUSY_sum", 0) / (256 * cyc),
              "mfma": a.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (1024 * cyc),
              "issue": a.get("SQ_ACTIVE_INST_ANY", 0) / (256 * cyc)}
        if m:
            ent["valu_mix_roof_frac_of_nominal"] = m["mix_roof_frac_of_nominal"]
            fr["valu_mix"] = a.get("SQ_INSTS_VALU", 0) * 2 / m["mix_roof_frac_of_nominal"] / (1024 * cyc)
        if a.get("SQ_INSTS_LDS"):
            ent["lds_conflict_per_instr"] = round(b.get("SQ_LDS_BANK_CONFLICT", 0) / a["SQ_INSTS_LDS"], 3)
        wc = b.get("SQ_WAVE_CYCLES", 0)
        if wc:
            ent["wave_wait_any_frac"] = round(b.get("SQ_WAIT_ANY", 0) / wc, 4)
            ent["wave_wait_inst_any_frac"] = round(b.get("SQ_WAIT_INST_ANY", 0) / wc, 4)
        ent["pipe_frac"] = {p: round(v, 4) for p, v in fr.items()}
        cand = {p: fr[p] for p in PIPES if p in fr}
        ent["binding_pipe"] = max(cand, key=cand.get)
        res["kernels"][k] = ent
    print(json.dumps(res, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
