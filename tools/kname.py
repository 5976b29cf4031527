"""Kernel-name keys for the profile tools: the full template instantiation of our kernels with
only the trailing parameter list dropped.

rocprofv3 reports demangled names such as
  void gs::raster_bwd3p_kernel<1, true, 16, true, float __vector(4)>(float const*, ...)
Cutting at the first '(' merges every instantiation whose template arguments hold a vector type
into one row (round 4's kernel-stats rows 2 and 4); this strips the balanced '(...)' at the end
instead, so each instantiation keeps its own key."""


def short_name(name):
    n = name.replace("(anonymous namespace)::", "")
    if not n.startswith(("void gs::", "gs::")):
        return n
    n = n.rstrip()
    if n.endswith(" [clone .kd]"):
        n = n[: -len(" [clone .kd]")]
    if not n.endswith(")"):
        return n
    depth = 0
    for i in range(len(n) - 1, -1, -1):
        c = n[i]
        if c == ")":
            depth += 1
        elif c == "(":
            depth -= 1
            if depth == 0:
                return n[:i]
    return n


if __name__ == "__main__":
    a = "void gs::raster_bwd3p_kernel<1, true, 16, true, float __vector(4)>(float const*, int)"
    b = "void gs::raster_bwd3p_kernel<1, true, 16, true, float __vector(2)>(float const*, int)"
    assert short_name(a) == "void gs::raster_bwd3p_kernel<1, true, 16, true, float __vector(4)>"
    assert short_name(a) != short_name(b)
    assert short_name("gs::(anonymous namespace)::k<3>(int)") == "gs::k<3>"
    print("ok")
