"""Copy the gzipped FileDescriptorProto blobs out of the reference's generated api.pb.go files
into tests/fixtures/reference_descriptors/ (see PROVENANCE.md there).

  python hack/extract_descriptors.py /root/reference
"""
import gzip
import hashlib
import os
import re
import sys

from google.protobuf import descriptor_pb2

SOURCES = {"deviceplugin_v1alpha": "pkg/kubelet/apis/deviceplugin/v1alpha/api.pb.go",
           "pluginregistration_v1beta": "pkg/kubelet/apis/pluginregistration/v1beta/api.pb.go",
           "cri_v1alpha1_runtime": "pkg/kubelet/apis/cri/v1alpha1/runtime/api.pb.go",
           "etcdserverpb_rpc": "vendor/github.com/coreos/etcd/etcdserver/etcdserverpb/rpc.pb.go",
           "mvccpb_kv": "vendor/github.com/coreos/etcd/mvcc/mvccpb/kv.pb.go"}
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "fixtures", "reference_descriptors")


def main(ref):
    for name, rel in SOURCES.items():
        text = open(os.path.join(ref, rel)).read()
        start = re.search(r"var fileDescriptor\w+ = \[\]byte\{", text).start()
        blob = bytes(int(h, 16) for h in re.findall(r"0x([0-9a-fA-F]{2})", text[start:text.index("\n}", start)]))
        descriptor_pb2.FileDescriptorProto.FromString(gzip.decompress(blob))    # must parse
        with open(os.path.join(OUT, name + ".pb.gz"), "wb") as f:
            f.write(blob)
        print(f"{name}: {rel}:{text[:start].count(chr(10)) + 1} {len(blob)} B sha256 {hashlib.sha256(blob).hexdigest()[:16]}")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference")
