"""Average / median duration (us) of the kernels in a rocprofv3 kernel-trace CSV whose name contains
each given substring.   python scripts/kt_avg.py trace.csv k_knn_rows k_knn_compact ..."""
import csv
import sys

import numpy as np

rows = list(csv.DictReader(open(sys.argv[1])))
for pat in sys.argv[2:]:
    d = np.array([(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows if pat in r["Kernel_Name"]])
    if len(d):
        print(f"{pat}: n {len(d)} mean {d.mean():.3f} median {np.median(d):.3f} us")
    else:
        print(f"{pat}: none")
