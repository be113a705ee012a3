package clients;

import com.google.protobuf.ByteString;
import inference.GRPCInferenceServiceGrpc;
import inference.GrpcService.InferTensorContents;
import inference.GrpcService.ModelInferRequest;
import inference.GrpcService.ModelInferResponse;
import inference.GrpcService.ServerLiveRequest;
import inference.GrpcService.ServerReadyRequest;
import io.grpc.ManagedChannel;
import io.grpc.ManagedChannelBuilder;
import java.nio.ByteBuffer;
import java.nio.ByteOrder;

/**
 * add/sub on "simple" through grpc-java stubs, with typed int_contents inputs
 * (reference src/grpc_generated/java/examples/.../SimpleJavaClient.java).
 *   mvn package && java -cp target/... clients.SimpleJavaClient localhost 8001
 */
public class SimpleJavaClient {
  public static void main(String[] args) {
    String host = args.length > 0 ? args[0] : "localhost";
    int port = args.length > 1 ? Integer.parseInt(args[1]) : 8001;
    ManagedChannel channel = ManagedChannelBuilder.forAddress(host, port).usePlaintext().build();
    GRPCInferenceServiceGrpc.GRPCInferenceServiceBlockingStub stub = GRPCInferenceServiceGrpc.newBlockingStub(channel);

    System.out.println("server live: " + stub.serverLive(ServerLiveRequest.getDefaultInstance()).getLive());
    System.out.println("server ready: " + stub.serverReady(ServerReadyRequest.getDefaultInstance()).getReady());

    InferTensorContents.Builder a = InferTensorContents.newBuilder();
    InferTensorContents.Builder b = InferTensorContents.newBuilder();
    for (int i = 0; i < 16; i++) {
      a.addIntContents(i);
      b.addIntContents(1);
    }
    ModelInferRequest req = ModelInferRequest.newBuilder()
        .setModelName("simple")
        .addInputs(ModelInferRequest.InferInputTensor.newBuilder()
                       .setName("INPUT0").setDatatype("INT32").addShape(1).addShape(16).setContents(a))
        .addInputs(ModelInferRequest.InferInputTensor.newBuilder()
                       .setName("INPUT1").setDatatype("INT32").addShape(1).addShape(16).setContents(b))
        .addOutputs(ModelInferRequest.InferRequestedOutputTensor.newBuilder().setName("OUTPUT0"))
        .addOutputs(ModelInferRequest.InferRequestedOutputTensor.newBuilder().setName("OUTPUT1"))
        .build();
    ModelInferResponse resp = stub.modelInfer(req);
    int[] sum = toInts(resp.getRawOutputContents(0));
    int[] diff = toInts(resp.getRawOutputContents(1));
    for (int i = 0; i < 16; i++) {
      System.out.printf("%d + 1 = %d; %d - 1 = %d%n", i, sum[i], i, diff[i]);
      if (sum[i] != i + 1 || diff[i] != i - 1) throw new IllegalStateException("incorrect result");
    }
    channel.shutdownNow();
    System.out.println("PASS: java grpc stub client");
  }

  private static int[] toInts(ByteString raw) {
    ByteBuffer bb = raw.asReadOnlyByteBuffer().order(ByteOrder.LITTLE_ENDIAN);
    int[] out = new int[bb.remaining() / 4];
    for (int i = 0; i < out.length; i++) out[i] = bb.getInt();
    return out;
  }
}
