package triton.client;

import triton.client.pojo.ResponseError;

/** Error reported by the server or raised by the client (reference InferenceException.java:34-39). */
public class InferenceException extends Exception {
  private final int status;

  public InferenceException(ResponseError err) { this(err.getError(), 0); }

  public InferenceException(String message) { this(message, 0); }

  public InferenceException(String message, int httpStatus) {
    super(message);
    this.status = httpStatus;
  }

  public InferenceException(Throwable cause) {
    super(cause);
    this.status = 0;
  }

  /** HTTP status of the failed request (0 when the error was raised client-side). */
  public int getStatus() { return status; }
}
