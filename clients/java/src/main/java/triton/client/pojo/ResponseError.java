package triton.client.pojo;

/** {"error": "..."} body of a failed request (reference pojo/ResponseError.java). */
public class ResponseError {
  private String error;

  public ResponseError() {}

  public ResponseError(String error) { this.error = error; }

  public String getError() { return error; }

  public void setError(String error) { this.error = error; }
}
