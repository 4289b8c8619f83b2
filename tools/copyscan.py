import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
names = [r["Kernel_Name"] for r in rows]
print("total", len(names), "copies", sum("copyBuffer" in n for n in names))
# print the kernel names around the first 6 copyBuffer occurrences after the first greedy_select
first_sel = next(i for i, n in enumerate(names) if "greedy_select" in n)
cnt = 0
for i in range(first_sel, len(names)):
    if "copyBuffer" in names[i]:
        print("---", i, [n[:50] for n in names[i-3:i+3]])
        cnt += 1
        if cnt > 8: break
# count copies between selects
import collections
between = collections.Counter()
last = None
c = 0
for n in names[first_sel:]:
    if "greedy_select" in n:
        between[c] += 1; c = 0
    elif "copyBuffer" in n:
        c += 1
print("copies between consecutive selects:", dict(between))
prev = collections.Counter()
for i, n in enumerate(names):
    if "copyBuffer" in n and i > 0 and "greedy_select" not in names[i - 1]:
        prev[names[i - 1][:70] + "  ->  " + names[i + 1][:40] if i + 1 < len(names) else ""] += 1
for k, v in prev.most_common(12):
    print(v, k)
# durations of copies
d = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows if "copyBuffer" in r["Kernel_Name"]]
d.sort()
print("copy us: median", d[len(d)//2] / 1e3, "max", d[-1] / 1e3, "sum", sum(d) / 1e3)
