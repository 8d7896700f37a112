"""Extracts the reference's proof test vectors into tests/golden/proof_fixture.json
(run in the build container, where /root/reference exists).

Source: pkg/proof/share_proof_test.go validShareProof() and
pkg/proof/row_proof_test.go validRowProof() / root — a ShareProof of one transaction
share ("1 transaction share" of pkg/proof/proof_test.go TestNewShareInclusionProof)
and its data root. Only the byte values are taken (data, not code)."""
import json
import os
import re

REF = "/root/reference/pkg/proof"
HERE = os.path.dirname(os.path.abspath(__file__))


def byte_lists(text):
    """Every innermost {0x.., ..} byte literal, in source order."""
    out = []
    for m in re.finditer(r"\{((?:\s*(?:0x[0-9a-fA-F]+|\d+)\s*,?)+)\}", text):
        out.append(bytes(int(x, 0) for x in re.findall(r"0x[0-9a-fA-F]+|\d+", m.group(1))))
    return out


def main():
    sp = open(os.path.join(REF, "share_proof_test.go")).read()
    rp = open(os.path.join(REF, "row_proof_test.go")).read()
    body = sp[sp.index("func validShareProof()"):]
    lists = byte_lists(body[:body.index("NamespaceId")])
    data, nodes = lists[0], lists[1:]
    ns_id = byte_lists(body[body.index("NamespaceId"):])[0]
    start = int(re.search(r"Start:\s*(\d+)", body).group(1))
    end = int(re.search(r"End:\s*(\d+)", body).group(1))
    root = byte_lists(rp[rp.index("var root"):])[0]
    vr = rp[rp.index("func validRowProof()"):]
    vr = vr[:vr.index("\n}\n")]
    row_roots = byte_lists(vr[vr.index("RowRoots"):vr.index("Proofs")])
    leaf_hash = byte_lists(vr[vr.index("LeafHash"):vr.index("Aunts")])[0]
    aunts = byte_lists(vr[vr.index("Aunts"):])
    fx = {
        "source": "pkg/proof/share_proof_test.go validShareProof, pkg/proof/row_proof_test.go validRowProof/root",
        "root": root.hex(),
        "share_proof": {"data": [data.hex()], "start": start, "end": end, "nodes": [n.hex() for n in nodes],
                        "namespace_id": ns_id.hex(), "namespace_version": 0},
        "row_proof": {"row_roots": [r.hex() for r in row_roots], "start_row": 0, "end_row": 0,
                      "proofs": [{"total": int(re.search(r"Total:\s*(\d+)", vr).group(1)),
                                  "index": int(re.search(r"Index:\s*(\d+)", vr).group(1)),
                                  "leaf_hash": leaf_hash.hex(), "aunts": [a.hex() for a in aunts]}]},
    }
    with open(os.path.join(HERE, "proof_fixture.json"), "w") as f:
        json.dump(fx, f, indent=1)
    print({k: (len(v) if isinstance(v, list) else v) for k, v in fx["share_proof"].items() if k != "data"},
          len(data), len(fx["row_proof"]["proofs"][0]["aunts"]))


if __name__ == "__main__":
    main()
