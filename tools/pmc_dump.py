#!/usr/bin/env python3
"""Print the counters of the last dispatch of each kernel matching argv[2] in a rocprofv3 --pmc output dir."""
import glob
import os
import sqlite3
import sys

d, pat = sys.argv[1], sys.argv[2]
for db in glob.glob(os.path.join(d, "**", "*.db"), recursive=True):
    c = sqlite3.connect(db)
    for (name,) in c.execute("select distinct kernel_name from counters_collection where kernel_name like ?", ("%" + pat + "%",)):
        last = c.execute("select max(dispatch_id) from counters_collection where kernel_name = ?", (name,)).fetchone()[0]
        print(name)
        for cn, v in c.execute("select counter_name, sum(value) from counters_collection where kernel_name = ? and "
                               "dispatch_id = ? group by counter_name", (name, last)):
            print("  %-24s %.4g" % (cn, v))
