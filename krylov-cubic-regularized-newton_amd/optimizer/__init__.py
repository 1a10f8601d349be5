"""Drop-in replacement of the reference's `optimizer` package
(Raymond30/Krylov-Cubic-Regularized-Newton, optimizer/*.py) whose Krylov-CRN
hot path runs on MI355X through libkrcn.  Put the directory that contains this
package first on sys.path and `from optimizer.loss import LogisticRegression`,
`from optimizer.cubic import Cubic_Krylov_LS` resolve here."""
