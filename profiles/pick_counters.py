"""Print the subset of the wanted PMC counters that `rocprofv3 -L` lists on this box.

    python profiles/pick_counters.py <rocprofv3 -L output> NAME [NAME ...]
"""
import re
import sys

text = open(sys.argv[1]).read()
have = set(re.findall(r"\b([A-Z][A-Z0-9_]+)\b", text))
print(" ".join(n for n in sys.argv[2:] if n in have))
