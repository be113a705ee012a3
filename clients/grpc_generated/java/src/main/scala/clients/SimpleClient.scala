package clients

import java.nio.{ByteBuffer, ByteOrder}

import inference.GRPCInferenceServiceGrpc
import inference.GrpcService.{InferTensorContents, ModelInferRequest, ServerLiveRequest, ServerReadyRequest}
import io.grpc.ManagedChannelBuilder

/** The same add/sub flow from Scala over the grpc-java stubs
  * (reference src/grpc_generated/java/examples/src/main/scala/clients/SimpleClient.scala).
  */
object SimpleClient {
  def main(args: Array[String]): Unit = {
    val host = if (args.length > 0) args(0) else "localhost"
    val port = if (args.length > 1) args(1).toInt else 8001
    val channel = ManagedChannelBuilder.forAddress(host, port).usePlaintext().build()
    val stub = GRPCInferenceServiceGrpc.newBlockingStub(channel)
    println(s"server live: ${stub.serverLive(ServerLiveRequest.getDefaultInstance).getLive}")
    println(s"server ready: ${stub.serverReady(ServerReadyRequest.getDefaultInstance).getReady}")

    def tensor(name: String, values: Seq[Int]) = {
      val c = InferTensorContents.newBuilder()
      values.foreach(v => c.addIntContents(v))
      ModelInferRequest.InferInputTensor.newBuilder()
        .setName(name).setDatatype("INT32").addShape(1).addShape(values.length).setContents(c)
    }
    val a = 0 until 16
    val b = Seq.fill(16)(1)
    val req = ModelInferRequest.newBuilder()
      .setModelName("simple")
      .addInputs(tensor("INPUT0", a))
      .addInputs(tensor("INPUT1", b))
      .addOutputs(ModelInferRequest.InferRequestedOutputTensor.newBuilder().setName("OUTPUT0"))
      .addOutputs(ModelInferRequest.InferRequestedOutputTensor.newBuilder().setName("OUTPUT1"))
      .build()
    val resp = stub.modelInfer(req)
    def ints(i: Int): Array[Int] = {
      val bb = resp.getRawOutputContents(i).asReadOnlyByteBuffer().order(ByteOrder.LITTLE_ENDIAN)
      Array.fill(bb.remaining() / 4)(bb.getInt())
    }
    val (sum, diff) = (ints(0), ints(1))
    for (i <- 0 until 16) {
      println(s"${a(i)} + ${b(i)} = ${sum(i)}; ${a(i)} - ${b(i)} = ${diff(i)}")
      require(sum(i) == a(i) + b(i) && diff(i) == a(i) - b(i), "incorrect result")
    }
    channel.shutdownNow()
    println("PASS: scala grpc stub client")
  }
}
