"""When did the host enqueue each kernel of one object's timed repetition, against when the GPU could have started it?
Reads a `rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv` run of tools/single_object_trace.py and
prints, per kernel of the last timed repetition: its start, the end of the kernel before it on the stream, and the end
of the host's launch call (same correlation id) -- a kernel whose launch call ends after its predecessor finished was
held back by the host, not by the GPU.  Tool only.

  python3 tools/launch_lag.py DIR/run_kernel_trace.csv DIR/run_hip_api_trace.csv
"""
import csv
import sys

sys.path.insert(0, __file__.rsplit("/", 2)[0] + "/tools")
from single_object_trace import AFTER_PASSES  # noqa: E402


def main(ktrace, atrace):
    rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], int(r["Correlation_Id"]))
                  for r in csv.DictReader(open(ktrace)))
    api = {}
    for r in csv.DictReader(open(atrace)):
        api[int(r["Correlation_Id"])] = (int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"])
    clears = [i for i, r in enumerate(rows) if "k_tsdf_clear" in r[2]]
    last = rows[clears[-AFTER_PASSES - 1]:clears[-AFTER_PASSES]]
    t0 = last[0][0]
    prev_end = None
    print(f"{'start':>9} {'prev_end':>9} {'launch_end':>10} {'host_late':>9}  kernel")
    for s, e, name, cid in last:
        a = api.get(cid)
        le = (a[1] - t0) / 1e3 if a else float("nan")
        pe = (prev_end - t0) / 1e3 if prev_end is not None else float("nan")
        late = le - pe if a and prev_end is not None else float("nan")
        print(f"{(s - t0) / 1e3:9.1f} {pe:9.1f} {le:10.1f} {late:9.1f}  {name.split('(')[0][:70]}")
        prev_end = e if prev_end is None else max(prev_end, e)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
