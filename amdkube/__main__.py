"""`python -m amdkube <component|kubectl> ...` (hyperkube equivalent, reference cmd/hyperkube)."""
import sys


def main():
    if len(sys.argv) < 2 or sys.argv[1] in ("-h", "--help"):
        from .cmd.components import COMPONENTS
        print("usage: python -m amdkube {kubectl," + ",".join(sorted(COMPONENTS)) + "} [flags]")
        return 0
    comp, argv = sys.argv[1], sys.argv[2:]
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
