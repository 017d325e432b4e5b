"""Embed device headers as C++ raw strings for hiprtc (jit.cpp): embed.py out.inc name=path..."""
import sys

out, pairs = sys.argv[1], sys.argv[2:]
with open(out, "w") as f:
    for pair in pairs:
        name, path = pair.split("=", 1)
        src = open(path).read()
        assert ")SPECRTC\"" not in src
        f.write(f'static const char {name}[] = R"SPECRTC({src})SPECRTC";\n')
