"""ugpu_dfa_plan_host: what ugpu_dfa_create would return and report (the
kernel a COUNT scan runs), decided on the host.  The drop-in matcher plans
every table this way and initialises a device only for an input it sends to
the GPU (integration/reflex_gpu_matcher.h eligible()).

CPU: the plan of known tables (prefiltered C2, xc C3, code-point runs C4,
anchored context walk, W with anchors rejected).  GPU: the plan equals
Pattern(...).info() of the uploaded tables over patterns x options W, N."""
import pytest

PATS = ["foo|bar|baz", "[A-Za-z_][A-Za-z0-9_]*", r"\w+", "a+", "^foo", "foo$", "x[a-z]*y", r"\d+\.\d+",
        "(ab)+", "[a-z]+ing", r"\S+", "[[:alpha:]]+", "é+", "a|b", ".", r"[0-9]{3}-[0-9]{4}", "a*"]


def test_plan_known_tables():
    import ugrep_amd as U
    assert U.host_plan("foo|bar|baz")["kernel"] == 0
    assert U.host_plan("[A-Za-z_][A-Za-z0-9_]*")["kernel"] == 5
    assert U.host_plan(r"\w+")["kernel"] == 6
    # line anchors / word boundaries: prefiltered tables run sparse_kernel's
    # context walks, the others wfind_kernel's chain of context walks
    assert U.host_plan("^foo")["kernel"] == 0
    assert U.host_plan("^foo", empty=True)["kernel"] == 0
    assert U.host_plan(r"\bfoo\b")["kernel"] == 0
    assert U.host_plan("^[a-z]+")["kernel"] == 4
    assert U.host_plan(r"\b[a-z]+\b")["kernel"] == 4
    with pytest.raises(U.Unsupported):
        U.host_plan("^foo", word=True)
    with pytest.raises(U.Unsupported):
        U.host_plan("a*", word=True, empty=True)


def test_plan_matches_host_tables():
    import ugrep_amd as U
    for rx in PATS:
        try:
            t = U.host_tables(U.compile_regex(rx))["info"]
        except U.Unsupported:
            continue
        p = U.host_plan(rx)
        for k in ("states", "classes", "row", "format", "table_bytes", "first_bytes", "accepting"):
            assert p[k] == t[k], (rx, k)


@pytest.mark.gpu
def test_plan_equals_uploaded_info():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a visible MI355X")
    import ugrep_amd as U
    for rx in PATS:
        for word in (False, True):
            for empty in (False, True):
                try:
                    plan = U.host_plan(rx, word=word, empty=empty)
                except U.Unsupported:
                    with pytest.raises(U.Unsupported):
                        U.Pattern(rx, word=word, empty=empty)
                    continue
                assert U.Pattern(rx, word=word, empty=empty).info() == plan, (rx, word, empty)
