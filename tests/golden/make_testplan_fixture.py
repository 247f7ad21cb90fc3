"""Extract the reference's bedops known-answer tests into a committed JSON fixture.

Source: applications/bed/bedops/test/TestPlan.xml (63 <TEST>s) run by
applications/bed/bedops/test/Regression.java. This script only reads the XML as
data (inputs, call, expected answer) and writes tests/golden/testplan.json with the
input files already expanded the way Regression.java writes them
(Regression.java:111-116 + updateString :179-196: every space removed, the
`chromosome` attribute + TAB prefixed to each non-empty line, '\n' after each line).

Run (in the build container, where /root/reference exists):
    python tests/golden/make_testplan_fixture.py /root/reference/applications/bed/bedops/test/TestPlan.xml
"""
import json
import os
import sys
import xml.etree.ElementTree as ET


def _expand(text, chrom):
    s = (text or "").strip().replace(" ", "")
    out = []
    for tok in s.split("\n"):
        if tok == "":  # java.util.StringTokenizer drops empty tokens
            continue
        out.append((chrom + "\t" if chrom else "") + tok + "\n")
    return "".join(out)


def main(path):
    root = ET.parse(path).getroot()
    tests = []
    for t in root.findall("TEST"):
        order = int(t.get("order"))
        chrom = t.get("chromosome") or ""
        call = ""
        inputs = []
        answer = ""
        output = None
        for child in t:
            if child.tag == "CALL":
                call += (child.text or "").strip()
            elif child.tag == "OUTPUT":
                output = child.get("name")
            elif child.tag == "INPUT":
                inputs.append({"name": child.get("name"), "data": _expand(child.text, chrom)})
            elif child.tag == "ANSWER":
                answer = _expand(child.text, chrom) if (child.text or "").strip() else ""
        tests.append({"order": order, "chromosome": chrom, "call": call.split(),
                      "inputs": inputs, "answer": answer, "output": output})
    tests.sort(key=lambda x: x["order"])
    dst = os.path.join(os.path.dirname(os.path.abspath(__file__)), "testplan.json")
    with open(dst, "w") as f:
        json.dump({"source": "applications/bed/bedops/test/TestPlan.xml", "tests": tests}, f, indent=1)
    print(f"wrote {len(tests)} tests to {dst}")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else
         "/root/reference/applications/bed/bedops/test/TestPlan.xml")
