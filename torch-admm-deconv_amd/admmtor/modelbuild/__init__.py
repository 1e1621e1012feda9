"""admmtor.modelbuild -- only the pieces of the reference's modelbuild that act on ADMMDeconv
(the parameter clamps).  The CNN models themselves are not part of this build."""
