"""Print per-kernel resource usage from a hipcc --cuda-device-only -S listing (probe helper)."""
import re
import sys

txt = open(sys.argv[1]).read()
for blk in re.split(r"\n\s+- \.(?=agpr_count|args)", txt):
    m = re.search(r"\.name:\s+(\S+)", blk)
    if not m:
        continue
    def g(k):
        r = re.search(r"\.%s:\s+(\d+)" % k, blk)
        return int(r.group(1)) if r else -1
    print(f"{m.group(1)[:70]:70s} vgpr={g('vgpr_count'):4d} agpr={g('agpr_count'):4d} "
          f"spill={g('private_segment_fixed_size'):4d} lds={g('group_segment_fixed_size')}")
