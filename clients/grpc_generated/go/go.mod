module github.com/triton-mi355x/client/examples

go 1.20

require (
	github.com/triton-mi355x/client/grpc-client v0.0.0
	google.golang.org/grpc v1.56.0
)

replace github.com/triton-mi355x/client/grpc-client => ./grpc-client
