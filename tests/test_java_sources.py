"""J1/J2/G2: static checks of the Java/Scala client sources (no JDK in the
build image, so they cannot be compiled here): token balance, package/path
and class/file agreement, intra-project imports resolve, and the API surface
of the reference Java subset is present."""

import os
import re

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
JAVA_ROOT = os.path.join(REPO, "clients", "java", "src", "main", "java")
STUB_ROOT = os.path.join(REPO, "clients", "grpc_generated", "java", "src", "main")


def _sources(root, ext):
    out = []
    for d, _, files in os.walk(root):
        out += [os.path.join(d, f) for f in files if f.endswith(ext)]
    return sorted(out)


def _strip(code):
    """Drop comments, string and char literals in one left-to-right pass
    (so "//" inside a string is not a comment)."""
    out, i, n = [], 0, len(code)
    while i < n:
        c = code[i]
        if code.startswith("//", i):
            j = code.find("\n", i)
            i = n if j < 0 else j
        elif code.startswith("/*", i):
            j = code.find("*/", i + 2)
            i = n if j < 0 else j + 2
        elif c in "\"'":
            j = i + 1
            while j < n and code[j] != c:
                j += 2 if code[j] == "\\" else 1
            out.append(c + c)
            i = j + 1
        else:
            out.append(c)
            i += 1
    return "".join(out)


ALL = _sources(JAVA_ROOT, ".java") + _sources(STUB_ROOT, ".java") + _sources(STUB_ROOT, ".scala")


@pytest.mark.parametrize("path", ALL, ids=lambda p: os.path.relpath(p, REPO))
def test_balanced(path):
    code = _strip(open(path).read())
    stack = []
    pairs = {")": "(", "]": "[", "}": "{"}
    for i, ch in enumerate(code):
        if ch in "([{":
            stack.append(ch)
        elif ch in ")]}":
            assert stack and stack[-1] == pairs[ch], "unbalanced %s at offset %d" % (ch, i)
            stack.pop()
    assert not stack, "unclosed %s" % stack


@pytest.mark.parametrize("path", _sources(JAVA_ROOT, ".java"), ids=lambda p: os.path.relpath(p, JAVA_ROOT))
def test_package_and_class_match_path(path):
    code = open(path).read()
    rel = os.path.relpath(os.path.dirname(path), JAVA_ROOT).replace(os.sep, ".")
    m = re.search(r"^package ([\w.]+);", code, re.M)
    assert m and m.group(1) == rel
    name = os.path.basename(path)[:-5]
    assert re.search(r"^public (?:final |abstract )?(?:class|enum|interface) %s\b" % name, code, re.M), name
    # every statement-level line inside a method ends sensibly (catch a missing ';')
    for ln in _strip(code).splitlines():
        s = ln.strip()
        if re.match(r"^(return|throw|int|long|double|float|String|byte\[\]|boolean)\b.*[\w)\]\"]$", s) and "(" not in s[-1:]:
            assert s.endswith((";", "{", ",", "(", "+", "&&", "||", "?", ":")) or s.endswith(")"), s


def test_project_imports_resolve():
    for path in _sources(JAVA_ROOT, ".java"):
        for imp in re.findall(r"^import (triton\.client[\w.]*);", open(path).read(), re.M):
            f = os.path.join(JAVA_ROOT, *imp.split(".")) + ".java"
            assert os.path.exists(f), "%s imports missing %s" % (path, imp)


def test_reference_api_surface():
    src = lambda n: open(os.path.join(JAVA_ROOT, "triton", "client", n)).read()
    inp = src("InferInput.java")
    for t in ("boolean", "byte", "short", "int", "long", "float", "double", "String"):
        assert "public void setData(%s[] data, boolean isBinaryData)" % t in inp, t
    res = src("InferResult.java")
    for t in ("Bool", "Byte", "Short", "Int", "Long", "Float", "Double", "String"):
        assert "getOutputAs%s(String output)" % t in res, t
    cli = src("InferenceServerClient.java")
    for m in ("public InferResult infer(InferArguments arg)", "public void setRetryCnt(int retryCnt)",
              "public InferArguments setSequenceId(long sequenceId)", "public InferArguments addQueryParam(",
              "public InferArguments setHeader(", "public CompletableFuture<InferResult> inferAsync(",
              "public static class HttpConfig"):
        assert m in cli, m
    from tritonclient.http import _utils  # noqa: F401  (wire constant shared with the Python client)

    assert '"Inference-Header-Content-Length"' in cli
    assert '"binary_data_output"' in cli and '"binary_data_size"' in src("pojo/Parameters.java")
    dt = src("pojo/DataType.java")
    for name in ("BOOL", "UINT8", "UINT16", "UINT32", "UINT64", "INT8", "INT16", "INT32", "INT64", "FP16", "BF16",
                 "FP32", "FP64", "BYTES"):
        assert re.search(r"\b%s\(" % name, dt), name


def test_examples_present():
    ex = os.path.join(JAVA_ROOT, "triton", "client", "examples")
    assert sorted(os.listdir(ex)) == ["MemoryGrowthTest.java", "SimpleInferClient.java", "SimpleInferPerf.java"]
