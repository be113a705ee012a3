package triton.client.endpoint;

/**
 * Source of the server address used for each request; subclasses can
 * implement discovery / load balancing (reference endpoint/AbstractEndpoint.java:39-60).
 */
public abstract class AbstractEndpoint {
  /** host:port (no scheme) of the server to send the next request to. */
  protected abstract String getEndpointImpl() throws Exception;

  /** Number of distinct endpoints; the client uses it to bound retries. */
  public abstract int getEndpointNum() throws Exception;

  public String getEndpoint() throws Exception {
    String ep = getEndpointImpl();
    if (ep == null || ep.isEmpty()) throw new IllegalStateException("endpoint is empty");
    return ep;
  }
}
