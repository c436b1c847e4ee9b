"""GPU busy vs idle time from a rocprofv3 kernel trace (csv): the union of the kernel intervals over
the traced span, the largest gaps, and the kernels just before / after them.

  python tools/gpu_idle.py kernel_trace.csv [first_kernel_substring_of_a_step]
"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
# skip the warm-up: start from the 3rd occurrence of the step marker kernel if given
if len(sys.argv) > 2:
    marks = [i for i, (_, _, n) in enumerate(iv) if sys.argv[2] in n]
    if len(marks) > 2:
        iv = iv[marks[2]:]
t0, t1 = iv[0][0], max(e for _, e, _ in iv)
busy, cur_s, cur_e = 0, iv[0][0], iv[0][1]
gaps = []
prev_name = iv[0][2]
for s, e, n in iv[1:]:
    if s > cur_e:
        busy += cur_e - cur_s
        gaps.append((s - cur_e, prev_name, n))
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
    prev_name = n
busy += cur_e - cur_s
span = t1 - t0
print(f"span {span / 1e6:.2f} ms, busy {busy / 1e6:.2f} ms, idle {(span - busy) / 1e6:.2f} ms "
      f"({100 * (span - busy) / span:.1f} %), {len(gaps)} gaps")
gaps.sort(reverse=True)
for g, a, b in gaps[:25]:
    print(f"  {g / 1e3:9.1f} us  after {a[:70]}  before {b[:70]}")
tot = {}
for g, a, b in gaps:
    k = b[:50]
    tot[k] = tot.get(k, 0) + g
print("idle by following kernel:")
for k, v in sorted(tot.items(), key=lambda kv: -kv[1])[:15]:
    print(f"  {v / 1e6:8.3f} ms  before {k}")
