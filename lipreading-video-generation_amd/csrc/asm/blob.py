"""Embed a code object as a C++ byte array: python blob.py IN.hsaco OUT.inc NAME"""
import sys

data = open(sys.argv[1], "rb").read()
name = sys.argv[3]
with open(sys.argv[2], "w") as f:
    f.write(f"// generated from {sys.argv[1].split('/')[-1]} by blob.py\n")
    f.write(f"alignas(4096) static const unsigned char {name}[{len(data)}] = {{\n")
    for i in range(0, len(data), 24):
        f.write("  " + ", ".join(str(b) for b in data[i:i + 24]) + ",\n")
    f.write("};\n")
