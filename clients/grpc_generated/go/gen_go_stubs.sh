#!/bin/bash
# Generate Go stubs for inference.GRPCInferenceService from this repo's protos
# (reference src/grpc_generated/go/gen_go_stubs.sh). Needs protoc,
# protoc-gen-go and protoc-gen-go-grpc on PATH.
set -euo pipefail
HERE="$(cd "$(dirname "$0")" && pwd)"
PROTO_DIR="${HERE}/../../../tritonclient/grpc/proto"
PACKAGE="github.com/triton-mi355x/client/grpc-client"
mkdir -p "${HERE}/grpc-client"
protoc -I "${PROTO_DIR}" \
  --go_out="${HERE}/grpc-client" --go_opt=paths=source_relative \
  --go_opt=Mgrpc_service.proto="${PACKAGE}" --go_opt=Mmodel_config.proto="${PACKAGE}" \
  --go-grpc_out="${HERE}/grpc-client" --go-grpc_opt=paths=source_relative \
  --go-grpc_opt=Mgrpc_service.proto="${PACKAGE}" --go-grpc_opt=Mmodel_config.proto="${PACKAGE}" \
  grpc_service.proto model_config.proto
echo "stubs written to ${HERE}/grpc-client"
