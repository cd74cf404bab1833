"""Regenerate tests/golden/reference_kats.json from the reference's own test files.

Run in the build container (where /root/reference exists):
    python tests/golden/make_golden.py [/root/reference]

Only numeric DATA is extracted (inputs/expected outputs the reference's tests
hold, located by test function and literal order); no reference source text
is stored.  Each entry records the file:function it came from.
"""
import ast
import json
import os
import sys

REF = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "reference_kats.json")


def _literals(path, func):
    """Numeric list literals (incl. np.array(...) / mi.Float(...) arguments) of one test function, in order."""
    tree = ast.parse(open(os.path.join(REF, path)).read())
    fn = next(n for n in ast.walk(tree) if isinstance(n, ast.FunctionDef) and n.name == func)
    out = []

    class V(ast.NodeVisitor):
        def visit_List(self, node):
            try:
                v = ast.literal_eval(node)
            except ValueError:
                return self.generic_visit(node)
            flat = json.dumps(v)
            if any(ch.isdigit() for ch in flat):
                out.append((node.lineno, v))

        def visit_UnaryOp(self, node):
            self.generic_visit(node)

    V().visit(fn)
    return out


def _calls(path, func, name):
    """(lineno, args, expected) of `assert dr.allclose(mi.<name>(...), expected)` style checks."""
    tree = ast.parse(open(os.path.join(REF, path)).read())
    fn = next(n for n in ast.walk(tree) if isinstance(n, ast.FunctionDef) and n.name == func)
    out = []
    for n in ast.walk(fn):
        if isinstance(n, ast.Compare) and isinstance(n.left, ast.Call):
            c = n.left
            if getattr(c.func, "attr", None) == name:
                try:
                    out.append((n.lineno, [ast.literal_eval(a) for a in c.args], ast.literal_eval(n.comparators[0])))
                except ValueError:
                    pass
    return sorted(out)


def main():
    kats = {}
    rnd = "src/core/tests/test_random.py"
    for f, name in (("test01_tea_float32", "sample_tea_float32"), ("test02_tea_float64", "sample_tea_float64")):
        kats[name] = {"source": "%s:%s" % (rnd, f),
                      "cases": [{"line": l, "v0": a[0], "v1": a[1], "rounds": a[2], "expected": e}
                                for l, a, e in _calls(rnd, f, name)]}

    mf = "src/render/tests/test_microfacet.py"
    lit = _literals(mf, "test02_eval_pdf_beckmann")
    tables = [v for _, v in lit if isinstance(v, list) and len(v) == 20]
    kats["beckmann_eval_pdf"] = {
        "source": mf + ":test02_eval_pdf_beckmann",
        "note": "theta sweep (0..pi, 20 steps, phi=pi/2) then phi sweep (theta=0.1); wi=(0,0,1); "
                "anisotropic alpha (0.1, 0.3) and isotropic 0.1, non-visible pdf",
        "theta_eval_aniso": tables[0], "theta_pdf_aniso": tables[1],
        "theta_eval_iso": tables[2], "theta_pdf_iso": tables[3],
        "phi_eval_aniso": tables[4], "phi_pdf_aniso_over_cos0.1": tables[5],
        "phi_eval_iso_const": 11.86709118}
    tree = ast.parse(open(os.path.join(REF, mf)).read())
    fns = [n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name == "test03_smith_g1_ggx"]
    for fn, key in ((next(n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name == "test03_smith_g1_beckmann"),
                     "beckmann_smith_g1"), (fns[0], "ggx_smith_g1")):
        vals = []
        for n in ast.walk(fn):
            if isinstance(n, ast.List):
                try:
                    v = ast.literal_eval(n)
                except ValueError:
                    continue
                if len(v) == 20:
                    vals.append((n.lineno, v))
        vals.sort()
        kats[key] = {"source": "%s:%s (line %d)" % (mf, fn.name, fn.lineno),
                     "note": "theta sweep pi/3..pi/2 (phi=pi/2): aniso (0.1,0.3), iso 0.1 (atol 1e-5); "
                             "phi sweep at theta=0.98*pi/2: aniso; iso constant = first aniso value",
                     "theta_aniso": vals[0][1], "theta_iso": vals[1][1], "phi_aniso": vals[2][1]}

    sen = "src/render/tests/test_sensor.py"
    kats["parse_fov"] = {"source": sen + ":test01_parse_fov", "cases": [
        {"focal_length": "50mm", "aspect": 0.5, "expected": 21.90213966369629},
        {"focal_length": "50mm", "aspect": 1.0, "expected": 34.02204132080078},
        {"focal_length": "50mm", "aspect": 1.5, "expected": 39.597713470458984},
        {"focal_length": "25mm", "aspect": 1.0, "expected": 62.923526763916016},
        {"fov": 35.0, "fov_axis": "diagonal", "aspect": 1.0, "expected": 25.137083053588867},
        {"fov": 35.0, "fov_axis": "y", "aspect": 0.5, "expected": 17.917831420898438},
        {"fov": 35.0, "fov_axis": "larger", "aspect": 0.5, "expected": 17.917831420898438},
        {"fov": 35.0, "fov_axis": "diagonal", "aspect": 0.5, "expected": 16.052263259887695},
        {"fov": 35.0, "fov_axis": "y", "aspect": 1.5, "expected": 50.6234245300293},
        {"fov": 35.0, "fov_axis": "smaller", "aspect": 1.5, "expected": 50.6234245300293},
        {"fov": 35.0, "fov_axis": "diagonal", "aspect": 1.5, "expected": 29.399948120117188},
        {"fov": 35.0, "fov_axis": "x", "aspect": 1.5, "expected": 35.0},
    ]}
    # cross-check the hand-listed expectations against the literal floats of the file
    src_floats = set()
    for n in ast.walk(ast.parse(open(os.path.join(REF, sen)).read())):
        if isinstance(n, ast.Constant) and isinstance(n.value, float):
            src_floats.add(n.value)
    for c in kats["parse_fov"]["cases"]:
        assert c["expected"] in src_floats, c
    pp = [v for _, v in _literals(sen, "test02_perspective_projection") if len(v) == 4 and isinstance(v[0], list)]
    kats["perspective_projection"] = {"source": sen + ":test02_perspective_projection",
                                      "film_size": [128, 32], "crop_size": [16, 8], "crop_offset": [8, 4],
                                      "fov_x": 35.0, "near": 10.0, "far": 1000.0, "matrix": pp[0]}
    for row in pp[0]:
        for x in row:
            assert abs(float(x)) in src_floats or float(x) in (0.0, 1.0), x
    json.dump(kats, open(OUT, "w"), indent=1)
    print("wrote", OUT, sorted(kats))


if __name__ == "__main__":
    main()
