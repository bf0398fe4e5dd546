"""Generate the golden fixtures in tests/golden/ from the reference's own test data.

Reads (as text only) the reference snapshot at /root/reference and writes
plain-data JSON fixtures: inputs and expected outputs, nothing else.

  * rs16_16_encode.json  <- src/tests/encode_data.zon + tests.zig:104-129
                            (RS(16,16), 64-B shards, input byte i % 256)
  * engine_kats.json     <- src/engines/Generic.zig:317-455
                            (ifftPartial x2, mulAdd, mul x4)

Run:  python tests/golden/make_fixtures.py [/root/reference]
The committed JSON files are what the tests read; the GPU box never needs
the reference.
"""
import json
import os
import re
import struct
import sys

REF = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


def nums(text):
    text = re.sub(r"\[\d+\]", "", text)          # drop array types like [2][64]
    text = re.sub(r"\b[ui]\d+\b", "", text)        # drop u8 / u64 type names
    return [int(t, 0) for t in re.findall(r"0x[0-9A-Fa-f]+|\d+", text)]


def lines(path, a, b):
    with open(os.path.join(REF, path)) as f:
        return "".join(f.readlines()[a - 1:b])


def u64s_to_bytes(vals):
    return list(struct.pack("<4Q", *vals))


def main():
    # ---- encode_data.zon: 16 x 64 parity bytes
    zon = open(os.path.join(REF, "src/tests/encode_data.zon")).read()
    parity = nums(zon)
    assert len(parity) == 16 * 64, len(parity)
    enc = {
        "source": "src/tests/encode_data.zon; src/tests.zig:104-129",
        "k": 16, "m": 16, "shard_bytes": 64,
        "input": "byte[i] = i % 256 over k*shard_bytes",
        "parity": [parity[i * 64:(i + 1) * 64] for i in range(16)],
    }
    with open(os.path.join(OUT, "rs16_16_encode.json"), "w") as f:
        json.dump(enc, f)

    g = "src/engines/Generic.zig"
    # ---- ifftPartial case 1 (Generic.zig:317-338)
    arr = nums(lines(g, 318, 328))
    assert len(arr) == 128, len(arr)
    # ---- ifftPartial case 2 (Generic.zig:340-368)
    inp2 = nums(lines(g, 341, 349))
    assert len(inp2) == 128, len(inp2)
    exp_x2 = nums(lines(g, 355, 365))
    assert len(exp_x2) == 128, len(exp_x2)
    assert "0xDDDD" in lines(g, 334, 334) and "0x4444" in lines(g, 354, 354)
    assert "0xE" in lines(g, 350, 350) and "0xE7" in lines(g, 350, 350)
    ifft_cases = [
        {"source": "Generic.zig:329-338", "log_m": 0xDDDD,
         "x": list(range(0, 128)), "y": list(range(128, 256)),
         "expected_x": arr, "expected_y": [128] * 128},
        {"source": "Generic.zig:340-368", "log_m": 0x4444,
         "x": arr, "y": inp2,
         "expected_x": exp_x2, "expected_y": ([0x0E] * 32 + [0xE7] * 32) * 2},
    ]
    # ---- mulAdd (Generic.zig:386-400)
    ma = lines(g, 386, 400)
    vecs = re.findall(r"Vector\(4, u64\)\{([^}]*)\}", ma)
    assert len(vecs) == 4, vecs
    v = [u64s_to_bytes(nums(x)) for x in vecs]
    assert "0x7777" in ma
    muladd = {"source": "Generic.zig:386-400", "log_m": 0x7777,
              "x_lo": v[0], "x_hi": v[1], "y_lo": [0x80] * 32, "y_hi": [0x80] * 32,
              "expected_lo": v[2], "expected_hi": v[3]}
    # ---- mul (Generic.zig:402-455)
    mul_text = lines(g, 402, 455)
    blocks = mul_text.split("const prod_lo, const prod_hi = mul(")[1:]
    mul_cases = []
    for b in blocks:
        splats = [int(x, 0) for x in re.findall(r"@splat\((0x[0-9A-Fa-f]+|\d+)\)", b)]
        lm = int(re.search(r"mul_128\[(0x[0-9A-Fa-f]+)\]", b).group(1), 16)
        assert len(splats) == 4, splats
        mul_cases.append({"lo": splats[0], "hi": splats[1], "log_m": lm,
                          "expected_lo": splats[2], "expected_hi": splats[3]})
    assert len(mul_cases) == 4
    kats = {"source": "src/engines/Generic.zig:317-455",
            "ifft_partial": ifft_cases, "mul_add": muladd, "mul": mul_cases}
    with open(os.path.join(OUT, "engine_kats.json"), "w") as f:
        json.dump(kats, f)
    print("wrote", os.listdir(OUT))


if __name__ == "__main__":
    main()
