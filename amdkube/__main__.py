"""`python -m amdkube <component|kubectl> ...` (hyperkube equivalent, reference cmd/hyperkube)."""
import os
import sys


def rootfs_paths(argv: list[str]) -> list[str]:
    """A process container without a mount namespace sees its volumes under $AMDKUBE_ROOTFS
    (runtime/rocshim.py links them there): an absolute path on the command line that exists in
    that view names the volume's file, which shadows the host's, as a mount would."""
    root = os.environ.get("AMDKUBE_ROOTFS")
    if not root:
        return argv

    def one(v: str) -> str:
        if v.startswith("/"):
            inside = os.path.join(root, v.lstrip("/"))
            if os.path.exists(inside):
                return inside
        return v
    out = []
    for arg in argv:
        if arg.startswith("--") and "=" in arg:
            k, v = arg.split("=", 1)
            out.append(f"{k}={one(v)}")
        else:
            out.append(one(arg))
    return out


def main():
    if len(sys.argv) < 2 or sys.argv[1] in ("-h", "--help"):
        from .cmd.components import COMPONENTS
        print("usage: python -m amdkube {kubectl," + ",".join(sorted(COMPONENTS)) + "} [flags]")
        return 0
    comp, argv = sys.argv[1], rootfs_paths(sys.argv[2:])
    if comp == "kubectl":
        from .kubectl.main import main as kubectl
        return kubectl(argv)
    from .cmd.components import COMPONENTS
    if comp not in COMPONENTS:
        print(f"unknown component {comp!r}", file=sys.stderr)
        return 2
    return COMPONENTS[comp](argv) or 0


if __name__ == "__main__":
    sys.exit(main())
