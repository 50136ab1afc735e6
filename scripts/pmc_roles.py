"""Per-role HBM traffic of a bench.py configuration from two rocprofv3 PMC passes (FETCH_SIZE,
WRITE_SIZE; scripts/gpu_run.sh pmc:...) over real forwards (bench.py --no-probe).

    python scripts/pmc_roles.py <root with FETCH_SIZE/ WRITE_SIZE/> <model> <dtype> <batch> <role>

Dispatches are attributed to the role by kernel name and, where two roles share one kernel
instantiation (out-proj and FC2 share the residual-LayerNorm epilogue), by their alternation
inside every encoder block (out-proj first). Traffic per launch = 2 x FETCH_SIZE (gfx950 tallies
128-B requests at 64 B: MI355X_MICROARCH.md, HBM) + WRITE_SIZE, averaged over the role's launches
(the same average as bench.py's per-role algorithmic bytes)."""
import csv
import datetime
import glob
import json
import os
import sys

# (model family, dtype) -> role -> [(kernel-name substring, modulus, remainder)]; rocprofv3
# demangles the float instantiations but not the bf16 (DF16b) ones of gemm_nt_kernel
RULES = {
    ("vit", "bf16"): {"fc1": [("gemm_pers_kernel<35,", 1, 0)],
                      # (4129 = LNIN | BIAS | HM: the head-major qkv store, round 5)
                      "qkv": [("gemm_pers_kernel<33,", 1, 0), ("gemm_pers_kernel<4129,", 1, 0)],
                      "out_proj": [("gemm_pers_kernel<197,", 2, 0), ("gemm_nt_kernelIDF16bLi197E", 2, 0)],
                      "fc2": [("gemm_pers_kernel<197,", 2, 1), ("gemm_nt_kernelIDF16bLi197E", 2, 1)],
                      "attention": [("attn_bf16_kernel", 1, 0)]},
    ("vit", "f32"): {"fc1": [("gemm_nt_kernel<float, 35>", 1, 0)],
                     "qkv": [("gemm_nt_kernel<float, 33>", 1, 0)],
                     "out_proj": [("gemm_nt_kernel<float, 197>", 2, 0)],
                     "fc2": [("gemm_nt_kernel<float, 197>", 2, 1)],
                     "attention": [("attn_f32_kernel", 1, 0)]},
    ("t2t", "bf16"): {"fc1": [("gemm_pers_kernel<35,", 1, 0)],
                      "qkv": [("gemm_pers_kernel<4129,", 1, 0)],  # head-major store (the kqv GEMMs are <33>)
                      "out_proj": [("gemm_pers_kernel<197,", 2, 0)],
                      "fc2": [("gemm_pers_kernel<197,", 2, 1)],
                      "attention": [("attn_bf16_kernel", 1, 0)]},
    ("swin", "bf16"): {"fc1": [("gemm_pers_kernel<289,", 1, 0), ("gemm_nt_kernelIDF16bLi289E", 1, 0)],
                       "out_proj": [("gemm_pers_kernel<133,", 2, 0), ("gemm_nt_kernelIDF16bLi133E", 2, 0)],
                       "fc2": [("gemm_pers_kernel<133,", 2, 1), ("gemm_nt_kernelIDF16bLi133E", 2, 1)],
                       "attention": [("window_attn_bf16_kernel", 1, 0)]},
}


def family(model):
    return "swin" if model.startswith("swin") else "t2t" if model.startswith("t2t") else "vit"


def rows_for(root, counter):
    f = glob.glob(os.path.join(root, counter, "**", "*counter_collection.csv"), recursive=True)
    rows = [r for r in csv.DictReader(open(f[0])) if r["Counter_Name"] == counter]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    return rows


def select(rows, rule):
    out = []
    for sub, mod, rem in rule:
        ks = [r for r in rows if sub in r["Kernel_Name"]]
        out += [r for i, r in enumerate(ks) if i % mod == rem]
    return out


def one(root, model, dtype, role):
    rule = RULES[(family(model), dtype)][role]
    f = select(rows_for(root, "FETCH_SIZE"), rule)
    w = select(rows_for(root, "WRITE_SIZE"), rule)
    assert f and len(f) == len(w), (len(f), len(w))
    fetch = 2 * 1024 * sum(float(r["Counter_Value"]) for r in f) / len(f)
    write = 1024 * sum(float(r["Counter_Value"]) for r in w) / len(w)
    return {"kernels": sorted({r["Kernel_Name"][:120] for r in f}), "launches": len(f),
            "fetch_bytes_corrected_per_launch": fetch, "write_bytes_per_launch": write,
            "traffic_bytes_per_launch": fetch + write}


def main():
    """<role> may be a comma-separated list: the first role's numbers stay at the top level, every
    role's under "roles" (bench.py looks its dominant role up there)."""
    root, model, dtype, batch, roles = sys.argv[1:6]
    roles = roles.split(",")
    per = {r: one(root, model, dtype, r) for r in roles}
    out = {"model": model, "dtype": dtype, "batch": int(batch), "role": roles[0], **per[roles[0]],
           "roles": per,
           "correction": "2 x FETCH_SIZE (gfx950: 128-B requests tallied at 64 B) + WRITE_SIZE",
           "commit": os.environ.get("COMMIT"),
           "collected": os.environ.get("COLLECTED") or datetime.datetime.utcnow().strftime("%Y-%m-%dT%H:%MZ")}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
