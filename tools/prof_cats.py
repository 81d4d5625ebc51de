"""GPU time of the last profiled step grouped by kernel family."""
import collections, csv, re, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "k_fe_spectrum" in r["Kernel_Name"]]
st = rows[starts[-2]:starts[-1]] if len(starts) > 1 else rows[starts[-1]:]
CATS = [("frontend", r"k_fe_|k_normalize_raw"), ("lstm", r"k_lstm"), ("conv", r"k_conv|k_sum_splits|k_bn_|k_col_partial"),
        ("heads", r"k_mfma|bf16_shadow"), ("mlp", r"k_sk_|k_ln_|k_colred|k_reduce_parts"), ("elbo", r"k_latent|k_output"),
        ("optim", r"k_adamw|k_sumsq|k_clip"), ("torch", r"at::native|rocclr")]
agg, cnt = collections.Counter(), collections.Counter()
for r in st:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    name = r["Kernel_Name"]
    cat = next((c for c, p in CATS if re.search(p, name)), "other:" + name[:40])
    agg[cat] += d; cnt[cat] += 1
for c, v in agg.most_common():
    print(f"{c:30s} {v:7.3f} ms {cnt[c]:5d} launches")
print(f"total {sum(agg.values()):.3f} ms {sum(cnt.values())} launches")
